set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# scheduler-strategy A/B of the f32 core: the same lab shapes (autotuned
# tiles), default build vs gemm.hip built with other LLVM scheduling strategies
for r in 1 2; do
for b in default max-ilp max-memory-clause; do
  [ -x labbin/gemm_lab_$b ] || continue
  timeout -k 10 300 ./labbin/gemm_lab_$b 20 > gpurun_out/lab_${b}_$r.jsonl 2> gpurun_out/lab_${b}_$r.err || exit 1
  echo "$b run $r: $(grep -c tflops gpurun_out/lab_${b}_$r.jsonl) shapes"
done
done

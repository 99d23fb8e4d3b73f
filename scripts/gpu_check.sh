#!/bin/bash
# GPU-box driver: runs named steps under their own time limits; stops at the
# first step that faults the GPU, aborts, segfaults or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name=$1; shift
  local secs=$1; shift
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if grep -qiE "memory access fault|illegal address|hipErrorIllegal|HSA_STATUS_ERROR|core dumped" "gpurun_out/$name.log"; then
    echo "GPU fault in $name: stopping"; exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"smoke tests bench"}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    groupby) run groupby 600 python -u -m pytest tests/test_groupby.py -x -v --timeout 120 --timeout-method thread ;;
    gbprof) export TMPDIR=/tmp; run gbprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/gbprof" -o run -- python scripts/groupby_profile.py ;;
    kernels) run kernels 900 python -m pytest tests/test_gpu_kernels.py -x -q ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-5} --warmup ${BENCH_WARMUP:-2} ${BENCH_ARGS:-} ;;
    benchsmall) run benchsmall 600 python bench.py --steps 3 --warmup 1 --rows 1000000 ;;
    prof) export TMPDIR=/tmp; run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python bench.py --steps 3 --warmup 1 ${BENCH_ARGS:-} ;;
    probe) run probe 600 python scripts/pcie_probe.py ;;
    prof_inception) export TMPDIR=/tmp; run prof_inception 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_inc" -o run -- python bench/configs.py inception --rows 1024 --steps 2 --warmup 1 ;;
    cfg_add) run cfg_add 600 python bench/configs.py add ;;
    cfg_reduce) run cfg_reduce 900 python bench/configs.py reduce ${CFG_ARGS:-} ;;
    cfg_inception) run cfg_inception 900 python bench/configs.py inception ${CFG_ARGS:-} ;;
    cfg_kmeans) run cfg_kmeans 600 python bench/configs.py kmeans ;;
    gpumodels) run gpumodels 900 python -m pytest tests/test_gpu_models.py -x -q ;;
    gemmbench) run gemmbench 600 python scripts/gemm_bench.py --json gpurun_out/gemm_bench.json ;;
    images) run images 600 python -m pytest tests/test_image_ops.py -x -q ;;
    ex_image) run ex_image 600 python examples/read_image.py --images 64 ;;
    examples) run examples 900 bash -c "python examples/quickstart.py && python examples/harmonic_mean.py && python examples/kmeans_demo.py" ;;
  esac
done
echo "all steps done"

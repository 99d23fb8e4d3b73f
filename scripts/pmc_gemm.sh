set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
i=0
for shape in "gemm 4096 4096 4096" "conv 2048 54 54 80 3 3 192 1 VALID" "conv 2048 12 12 768 1 1 192 1 SAME" "conv 2048 109 109 32 3 3 64 1 SAME"; do
  i=$((i+1))
  timeout -k 5 120 python scripts/gemm_one.py $shape --iters 10 > gpurun_out/pmc/t$i.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $PWD/gpurun_out/pmc/p$i -o run -- python scripts/gemm_one.py $shape --iters 3 > gpurun_out/pmc/p$i.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d $PWD/gpurun_out/pmc/q$i -o run -- python scripts/gemm_one.py $shape --iters 3 > gpurun_out/pmc/q$i.log 2>&1 || exit 1
done
cat gpurun_out/pmc/t*.log | grep '{'

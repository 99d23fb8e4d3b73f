set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prec.log 2>&1; tail -1 gpurun_out/prec.log
SHAPES=scripts/tile_ab_r4e.txt TILES="auto 13 20 21" timeout -k 10 900 bash scripts/tile_ab.sh > gpurun_out/tile_ab_r4e.log 2>&1; grep -c tflops gpurun_out/tile_ab_r4e.log

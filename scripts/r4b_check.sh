set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=smoke bash scripts/gpu_check.sh &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool_accounting.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pooltest.log 2>&1; tail -3 gpurun_out/pooltest.log
STEPS=r4_kmeans bash scripts/gpu_steps.sh && STEPS="incep1m_u8 tests" bash scripts/gpu_steps.sh

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_engine.py tests/test_groupby.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kern.log 2>&1; tail -2 gpurun_out/kern.log
STEPS=r4_kmeans bash scripts/gpu_steps.sh

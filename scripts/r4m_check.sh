set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=smoke bash scripts/gpu_check.sh && STEPS="tests bench incep_dev" bash scripts/gpu_steps.sh
TFA_GEMM_TUNE_LOG=1 timeout -k 10 120 python scripts/gemm_one.py gemm 4096 4096 4096 --iters 30 > gpurun_out/g4096.log 2>&1; grep -v amdgpu gpurun_out/g4096.log

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=smoke bash scripts/gpu_check.sh && STEPS=tests bash scripts/gpu_steps.sh

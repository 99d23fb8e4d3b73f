set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="smoke tests incep_dev bench" bash scripts/gpu_steps.sh

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPES=scripts/tile_ab_r4d.txt TILES="auto 16 8 6 21" timeout -k 10 900 bash scripts/tile_ab.sh > gpurun_out/tile_ab_r4d.log 2>&1; grep -c tflops gpurun_out/tile_ab_r4d.log
STEPS=incep_dev bash scripts/gpu_steps.sh

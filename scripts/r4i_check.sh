set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
STEPS=prof_incep bash scripts/gpu_steps.sh
OUT=gpurun_out/pmc_r4t SHAPES="c4a16|conv 52x52 3x3 80->192 (Conv2d_4a, 128x192 8-wave)|16|gemm_f32_tile|conv 2048 54 54 80 3 3 192 1 VALID
c4a8|conv 52x52 3x3 80->192 (Conv2d_4a, 64x192 4-wave)|8|gemm_f32_tile|conv 2048 54 54 80 3 3 192 1 VALID" timeout -k 10 600 bash scripts/pmc_gemm.sh > gpurun_out/pmc_r4t.log 2>&1; tail -8 gpurun_out/pmc_r4t.log

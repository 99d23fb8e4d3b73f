#!/bin/bash
# round 5: counters of the g2 core (library tile 22, B^T) against the g2 lab
# kernel (MODE 3) and the round-4 core (tile 21) on 4096^3, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/g2_lab.hip -o /tmp/g2_lab || exit 3
timeout -k 10 120 /tmp/g2_lab 4096 4096 4096 > "$OUT/lab_time.log" 2>&1 || exit 1
cat "$OUT/lab_time.log"
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $PA --output-format csv -d "$PWD/$OUT/laba" -o run -- /tmp/g2_lab 4096 4096 4096 one > "$OUT/laba.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $PB --output-format csv -d "$PWD/$OUT/labb" -o run -- /tmp/g2_lab 4096 4096 4096 one > "$OUT/labb.log" 2>&1 || exit 1
SHAPES="t22tb|gemm 4096^3 B^T (g2 256x256)|22|g2_tile|gemm 4096 4096 4096 --tb
t22|gemm 4096^3 (g2 256x256, B [K][N])|22|g2_tile|gemm 4096 4096 4096
t21|gemm 4096^3 (round-4 256x256)|21|gemm_f32_tile|gemm 4096 4096 4096
c4a23|Conv2d_4a (g2 256x192)|23|g2_tile|conv 2048 54 54 80 3 3 192 1 VALID
c4a16|Conv2d_4a (round-4 tile 16)|16|gemm_f32_tile|conv 2048 54 54 80 3 3 192 1 VALID" OUT=$OUT bash scripts/pmc_gemm.sh

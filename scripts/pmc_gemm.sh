#!/bin/bash
# rocprofv3 --pmc of the f32 GEMM / implicit-GEMM conv core on fixed shapes
# with forced tiles (TFA_GEMM_TILE), two counter passes per shape, each in its
# own run; summary: python scripts/pmc_summary.py $OUT
#   OUT=gpurun_out/pmc4 bash scripts/pmc_gemm.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/pmc4}
mkdir -p "$OUT"
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
# id|name|tile|kernel match|gemm_one args
SHAPES=${SHAPES:-"g4096|gemm 4096^3 (256x128 8-wave)|13|gemm_f32_tile|gemm 4096 4096 4096
c4a|conv 52x52 3x3 80->192 (Conv2d_4a, 64x192)|8|gemm_f32_tile|conv 2048 54 54 80 3 3 192 1 VALID
c6pw|conv 12x12 1x1 768->192 (64x192)|8|gemm_f32_tile|conv 2048 12 12 768 1 1 192 1 SAME
c3b|gemm 5.97M x 80 x 64 (Conv2d_3b, 256x96 8-wave)|14|gemm_f32_tile|gemm 5971968 80 64
c6a|conv 25x25 3x3/2 288->384 (Mixed_6a, 128x128 2x4)|15|gemm_f32_tile|conv 2048 25 25 288 3 3 384 2 VALID"}
echo "[" > "$OUT/shapes.json"
first=1
while IFS='|' read -r id name tile kern args; do
  [ -z "$id" ] && continue
  [ $first = 1 ] || echo "," >> "$OUT/shapes.json"
  first=0
  printf '{"id": "%s", "name": "%s", "tile": %s, "kernel": "%s"}' "$id" "$name" "$tile" "$kern" >> "$OUT/shapes.json"
  echo "== $id ($(date +%T))"
  TFA_GEMM_TILE=$tile timeout -k 5 120 python scripts/gemm_one.py $args --iters 10 > "$OUT/${id}t.log" 2>&1 || exit 1
  grep '{' "$OUT/${id}t.log"
  TFA_GEMM_TILE=$tile timeout -s KILL 90 rocprofv3 --pmc $PA --output-format csv -d "$PWD/$OUT/${id}a" -o run -- python scripts/gemm_one.py $args --iters 3 > "$OUT/${id}a.log" 2>&1 || exit 1
  TFA_GEMM_TILE=$tile timeout -s KILL 90 rocprofv3 --pmc $PB --output-format csv -d "$PWD/$OUT/${id}b" -o run -- python scripts/gemm_one.py $args --iters 3 > "$OUT/${id}b.log" 2>&1 || exit 1
done <<< "$SHAPES"
echo "]" >> "$OUT/shapes.json"
python scripts/pmc_summary.py "$OUT" | tee "$OUT/summary.md"

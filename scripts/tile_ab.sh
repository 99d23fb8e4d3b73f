#!/bin/bash
# GPU box: one shape per line through scripts/gemm_one.py under each forced
# f32 tile (TFA_GEMM_TILE), plus the autotuned default; prints TF/s.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TILES=${TILES:-"auto 0 6 9 10 12 13 14 15 16"}
while read -r shape; do
  [ -z "$shape" ] && continue
  for t in $TILES; do
    if [ "$t" = auto ]; then
      TFA_GEMM_TUNE_LOG=1 timeout -k 5 120 python scripts/gemm_one.py $shape --iters 30 2>&1 | grep -E "gemm tune|kind" || exit 1
    else
      TFA_GEMM_TILE=$t timeout -k 5 120 python scripts/gemm_one.py $shape --iters 30 || exit 1
    fi
  done
done < "${SHAPES:-scripts/tile_ab_shapes.txt}"

#!/bin/bash
# GPU box: build the g2 GEMM lab and compare it with the shipped f32 core on
# the same shapes (each step under its own limit; stop at the first fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lab
OUT=gpurun_out/lab
hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/g2_lab.hip -o /tmp/g2_lab || exit 3
for shape in ${G2_SHAPES:-"4096 4096 4096" "8192 8192 8192" "5537792 192 720" "2560000 512 512" "1280000 64 1200"}; do
  echo "== g2 $shape"
  timeout -k 10 120 /tmp/g2_lab $shape | tee -a $OUT/g2.jsonl; rc=$?
  [ $rc -ne 0 ] && { echo "g2 rc=$rc: stopping"; exit $rc; }
done
for shape in ${SHIPPED:-}; do
  echo "== shipped gemm $shape"
  timeout -k 10 180 python scripts/gemm_one.py gemm $shape --iters 20 | tee -a $OUT/shipped.log; rc=$?
  [ $rc -ne 0 ] && { echo "shipped rc=$rc: stopping"; exit $rc; }
done
exit 0

#!/bin/bash
# round 5: g2 core correctness on the GPU (fp64 reference + bitwise tile
# invariance), then kernel-level A/B against the round-4 core (forced tiles)
# on 4096^3 / 8192^3, the headline 2.5M x 512 x 512 and Inception Conv2d_4a.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/r5/$name.log"
  if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|core dumped" "gpurun_out/r5/$name.log"; then
    echo "GPU fault in $name"; exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; exit $rc; fi
}
step g2_tests 400 python -u -m pytest tests/test_gpu_g2.py tests/test_gpu_precision.py -x -q --timeout 300 --timeout-method thread
for t in ${TILES:-21 22 23 24}; do
  TFA_GEMM_TILE=$t step "ab_4096_t$t" 120 python scripts/gemm_one.py gemm 4096 4096 4096 --iters 30
  TFA_GEMM_TILE=$t step "ab_4096tb_t$t" 120 python scripts/gemm_one.py gemm 4096 4096 4096 --iters 30 --tb
  TFA_GEMM_TILE=$t step "ab_8192_t$t" 120 python scripts/gemm_one.py gemm 8192 8192 8192 --iters 10
done
for t in ${HEAD_TILES:-13 22 23 24 25}; do
  TFA_GEMM_TILE=$t step "ab_head_t$t" 120 python scripts/gemm_one.py gemm 2500000 512 512 --iters 20
done
for t in ${CONV_TILES:-16 23 24 25 26}; do
  TFA_GEMM_TILE=$t step "ab_conv4a_t$t" 120 python scripts/gemm_one.py conv 2048 54 54 80 3 3 192 1 VALID --iters 10
done
[ -n "${SKIP_BENCH:-}" ] && exit 0
step bench 300 python bench.py
step incep_dev 600 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1
exit 0

#!/bin/bash
# round 5: forced-tile A/B of single shapes (gemm_one.py): AB="name|tiles|args;..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5/ab  # (scripts/gpu_steps.sh step `ab`)
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/ab/tests.log 2>&1 || { tail -20 gpurun_out/r5/ab/tests.log; exit 1; }
  tail -2 gpurun_out/r5/ab/tests.log
fi
IFS=';' read -ra items <<< "$AB"
for it in "${items[@]}"; do
  IFS='|' read -r name tiles args <<< "$it"
  for t in $tiles; do
    TFA_GEMM_TILE=$t timeout -k 10 120 python scripts/gemm_one.py $args --iters 10 > gpurun_out/r5/ab/${name}_t$t.log 2>&1
    rc=$?
    if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|core dumped" gpurun_out/r5/ab/${name}_t$t.log; then echo "GPU fault"; exit 99; fi
    [ $rc -ne 0 ] && { echo "$name t$t rc=$rc"; tail -3 gpurun_out/r5/ab/${name}_t$t.log; exit $rc; }
    echo "$name t$t $(grep -o '"tflops": [0-9.]*' gpurun_out/r5/ab/${name}_t$t.log)"
  done
done
exit 0

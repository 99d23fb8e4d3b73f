#!/bin/bash
# round 5: batched image pre-stage (tests + read_image example), then the g2 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5/$name.log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/r5/$name.log"
  if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|core dumped" "gpurun_out/r5/$name.log"; then
    echo "GPU fault in $name"; exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; exit $rc; fi
}
step img_tests 300 python -u -m pytest tests/test_gpu_image_prep.py -x -v --timeout 200 --timeout-method thread
step read_image 600 python examples/read_image.py --images 2048
TFA_MAP_ROWS_BATCHED_PRESTAGE=0 step read_image_perrow 600 python examples/read_image.py --images 2048
exit 0

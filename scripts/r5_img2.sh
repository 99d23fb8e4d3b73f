#!/bin/bash
# round 5: where the image-scoring time goes (decode threads, GPU kernel time)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/r5/$name.log"
  if grep -qiE "memory access fault|illegal address|HSA_STATUS_ERROR|core dumped" "gpurun_out/r5/$name.log"; then
    echo "GPU fault in $name"; exit 99
  fi
  if [ $rc -ne 0 ]; then echo "stop after $name rc=$rc"; exit $rc; fi
}
step decode_bench 300 python scripts/decode_bench.py --images 1024
for t in 8 16; do
  TFA_DECODE_THREADS=$t step read_image_t$t 400 python examples/read_image.py --images 2048
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step read_image_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof_img -o img -- python3 examples/read_image.py --images 2048
exit 0

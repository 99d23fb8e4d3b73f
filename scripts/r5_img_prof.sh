#!/bin/bash
# round 5: where the steady-state image-scoring time goes (host profile, GPU kernel stats)
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
step img_cprofile 400 python -m cProfile -o gpurun_out/r5/img.prof examples/read_image.py --images 4096
export TMPDIR=/tmp
step img_rocprof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_img -o img -- python3 examples/read_image.py --images 4096
exit 0

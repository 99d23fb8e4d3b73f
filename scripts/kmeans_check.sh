#!/bin/bash
# GPU box: K-Means (in-graph variant) kernels per iteration, ms/iteration and
# a host-side cProfile of the iteration loop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/kmeans
mkdir -p $out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for it in 2 12; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/i${it} -o run -- \
    python scripts/kmeans_profile.py --iters $it > $out/i${it}.log 2>&1 || { echo "kmeans prof i$it failed"; tail -20 $out/i${it}.log; exit 1; }
done
timeout -k 10 240 python scripts/kmeans_profile.py --iters 20 > $out/timing.log 2>&1 || exit 1
timeout -k 10 240 python scripts/kmeans_profile.py --iters 10 --variant aggregate >> $out/timing.log 2>&1 || exit 1
timeout -k 10 240 python scripts/kmeans_profile.py --iters 20 --cprofile > $out/cprofile.log 2>&1 || exit 1
grep '{' $out/timing.log

#!/bin/bash
# GPU box: fusion numerics + K-Means kernel counts with fusion off/on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fusion
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for mode in 0 1; do
  for it in 2 12; do
    TFA_FUSION=$mode timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/fusion/f${mode}_i${it} -o run -- python scripts/kmeans_profile.py --iters $it \
      > gpurun_out/fusion/f${mode}_i${it}.log 2>&1 || { echo "kmeans prof f$mode i$it failed"; tail -20 gpurun_out/fusion/f${mode}_i${it}.log; exit 1; }
    grep '{' gpurun_out/fusion/f${mode}_i${it}.log
  done
done
for mode in 0 1; do
  TFA_FUSION=$mode timeout -k 10 240 python scripts/kmeans_profile.py --iters 20 --variant in_graph >> gpurun_out/fusion/timing.log 2>&1 || exit 1
  TFA_FUSION=$mode timeout -k 10 240 python scripts/kmeans_profile.py --iters 10 --variant aggregate >> gpurun_out/fusion/timing.log 2>&1 || exit 1
done
grep '{' gpurun_out/fusion/timing.log

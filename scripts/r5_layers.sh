#!/bin/bash
# round 5: the per-layer Inception-v3 conv table (ms, TF/s, tile, MFMA busy,
# VALU/MFMA) on the final kernels -> gpurun_out/r5/layers/
#   PART=time | PART="pmc FIRST LAST"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5/layers
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -- ${PART:-time}
if [ "$1" = time ]; then
  timeout -k 10 600 python scripts/conv_layers.py --json gpurun_out/r5/layers/layers.json > gpurun_out/r5/layers/conv_layers.log 2>&1
  rc=$?; tail -18 gpurun_out/r5/layers/conv_layers.log; exit $rc
fi
timeout -k 10 1100 python scripts/layers_pmc.py --layers scripts/data/inception_layers.json --out gpurun_out/r5/layers --first $2 --last $3 > gpurun_out/r5/layers/pmc_$2.log 2>&1
rc=$?; tail -3 gpurun_out/r5/layers/pmc_$2.log; exit $rc

#!/bin/bash
# round 5: pool accounting (1 rank and 2 ranks on the GPU), engine fills
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool_accounting.py tests/test_multirank_gpu.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/misc_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5/misc_tests.log; exit $rc

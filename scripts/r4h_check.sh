set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TFA_CONCURRENT_PARTITIONS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_models.py tests/test_gpu_pool_accounting.py -x -q --timeout 200 --timeout-method thread > gpurun_out/conc_tests1.log 2>&1; tail -1 gpurun_out/conc_tests1.log
for m in 0 1 0 1 0 1; do TFA_CONCURRENT_PARTITIONS=$m timeout -k 10 120 python scripts/kmeans_profile.py --iters 300 2>/dev/null | cut -c1-70 | sed "s/^{/{\"conc\": $m, /"; done
for m in 0 1 0 1; do TFA_CONCURRENT_PARTITIONS=$m timeout -k 10 120 python scripts/kmeans_profile.py --iters 200 --variant aggregate 2>/dev/null | cut -c1-70 | sed "s/^{/{\"conc\": $m, /"; done
TFA_CONCURRENT_PARTITIONS=1 timeout -k 10 120 python scripts/kmeans_phases.py --iters 300 2>/dev/null

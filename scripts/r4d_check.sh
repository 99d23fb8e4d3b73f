set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_plan_reuse.py tests/test_gpu_models.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/reuse.log 2>&1; tail -2 gpurun_out/reuse.log
timeout -k 10 300 python scripts/kmeans_host_parts.py --iters 300 > gpurun_out/khost.log 2>&1; head -22 gpurun_out/khost.log
TFA_PLAN_TIMING=3 timeout -k 10 120 python scripts/kmeans_profile.py --iters 20 > gpurun_out/kreb.log 2>&1; grep "tfa rebind" gpurun_out/kreb.log | tail -3
STEPS=r4_kmeans bash scripts/gpu_steps.sh > /dev/null 2>&1; cat gpurun_out/r4_kmeans/in_graph.log gpurun_out/r4_kmeans/aggregate.log gpurun_out/r4_kmeans/phases.log

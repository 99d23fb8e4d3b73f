"""Two ranks sharing the one GPU (gloo for the cross-rank exchange, since RCCL
refuses two ranks on a device): device-resident reduce_blocks, aggregate key
routing, groupBy count, long string keys, repartition and K-Means agree with
numpy, and every device temporary of both ranks came from the engine pool
(no fallbacks; scripts/multirank_rehearsal.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_two_ranks_on_one_gpu_match_numpy():
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import launch
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env["TFA_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(launch.free_port()),
                        os.path.join(REPO, "scripts", "multirank_rehearsal.py")],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=100)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["ok"] and out["world"] == 2, out
    assert out["pool_fallbacks"] == 0, out

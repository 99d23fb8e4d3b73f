"""An allocation neither the engine pool nor the framework allocator can
serve raises torch.OutOfMemoryError instead of deadlocking: the pool drops
its lock before falling back to at::empty, whose OOM observer
(dev_pool_install_oom_hook) takes the same lock (csrc/runtime/device_pool.cpp;
round-4 ADVICE high #1). Runs in a child process under a time limit, so a
regression shows as a timeout, not a hung suite."""
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

CODE = r"""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from tensorframes_amd import engine
from tensorframes_amd._native import _C
small = engine.device_empty((1 << 20,), torch.float32, "cuda:0")  # the pool works
try:
    engine.device_empty((1 << 42,), torch.float32, "cuda:0")      # 16 TiB: no allocator can serve it
    print("NO-ERROR")
except torch.OutOfMemoryError:
    print("OOM-RAISED", _C.device_pool_stats()["fallbacks"])
again = engine.device_empty((1 << 20,), torch.float32, "cuda:0")  # and the pool still works after it
torch.cuda.synchronize()
print("ALIVE")
"""


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_double_oom_raises_instead_of_deadlocking():
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", CODE], cwd=repo, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "OOM-RAISED" in p.stdout and "ALIVE" in p.stdout, p.stdout + p.stderr[-2000:]

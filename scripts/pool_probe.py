"""Device-pool probe: per-call cost of a tiny device program (x + 1) and the
K-Means iteration, with the pool's counters (reuse vs fresh hipMalloc)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402

dev = torch.device("cuda", 0)
g = tf.Graph()
with g.as_default():
    x = tf.placeholder(tf.float32, [None, 16], name="x")
    tf.add(x, 1.0, name="y")
prog = engine.program(g.serialize(), ["y"], ["x"])
xin = torch.rand(1024, 16, device=dev)
for _ in range(100):
    engine.run_program(prog, [xin], dev)
torch.cuda.synchronize()
s0 = _C.device_pool_stats()
t0 = time.perf_counter()
for _ in range(5000):
    engine.run_program(prog, [xin], dev)
torch.cuda.synchronize()
t1 = time.perf_counter()
s1 = _C.device_pool_stats()
rng = np.random.default_rng(2)
pts = rng.uniform(0.0, 1.0, size=(100_000, 100))
df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4)).cache_on_device(dev)
c = np.random.default_rng(2).standard_normal((10, 100))
kmeans.kmeans(df, c, num_iters=2)
torch.cuda.synchronize()
s2 = _C.device_pool_stats()
t2 = time.perf_counter()
for _ in range(30):
    c, _d = kmeans.run_one_step2(df, c)
torch.cuda.synchronize()
t3 = time.perf_counter()
s3 = _C.device_pool_stats()
print(json.dumps({"pool": os.environ.get("TFA_DEVICE_POOL", "1"), "tiny_us_per_run": (t1 - t0) / 5000 * 1e6,
                  "tiny_pool_delta": {k: s1[k] - s0[k] for k in s1},
                  "kmeans_ms_per_iter": (t3 - t2) / 30 * 1e3,
                  "kmeans_pool_delta": {k: s3[k] - s2[k] for k in s3}}))

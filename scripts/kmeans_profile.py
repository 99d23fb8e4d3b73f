"""K-Means (reference demo shape: 100k points x 100 features, k=10) on a
device-cached frame: prints ms/iteration for the in-graph (map_blocks +
reduce_blocks) and aggregate variants. Run under rocprofv3 with
--iters 2 and --iters 12 to get kernels per iteration from the difference."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--variant", choices=["in_graph", "aggregate"], default="in_graph")
ap.add_argument("--points", type=int, default=100_000)
ap.add_argument("--cprofile", action="store_true", help="print the top host functions by own time")
a = ap.parse_args()
rng = np.random.default_rng(2)
pts = rng.uniform(0.0, 1.0, size=(a.points, 100))
df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4)).cache_on_device(engine.compute_device())
c0 = np.random.default_rng(2).standard_normal((10, 100))
agg = a.variant == "in_graph"
for _ in range(5):  # warm: plans, JIT, tile tuning, HIP-graph captures of the per-partition runs
    (kmeans.run_one_step2 if agg else kmeans.run_one_step)(df, c0)
torch.cuda.synchronize() if torch.cuda.is_available() else None
prof = None
if a.cprofile:
    import cProfile
    prof = cProfile.Profile()
    prof.enable()
t0 = time.perf_counter()
c = c0
for _ in range(a.iters):
    c, _d = (kmeans.run_one_step2 if agg else kmeans.run_one_step)(df, c)
torch.cuda.synchronize() if torch.cuda.is_available() else None
dt = (time.perf_counter() - t0) / a.iters
if prof is not None:
    import pstats
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    pstats.Stats(prof).sort_stats("cumulative").print_stats(60)
from tensorframes_amd._native import _C  # noqa: E402
graphs = {}
for p in list(engine._prog_cache.values()):
    for k in ("graphs_captured", "graph_replays", "graphs_declined", "runs"):
        graphs[k] = graphs.get(k, 0) + p.stats()[k]
print(json.dumps({"variant": a.variant, "iters": a.iters, "ms_per_iter": dt * 1e3,
                  "fusion": os.environ.get("TFA_FUSION", "1"), "jit": _C.jit_stats(), "programs": graphs}))

"""Wall-clock breakdown of one K-Means iteration (run_one_step2, 100k x 100 f64,
k = 10, device-cached): timers wrapped around the framework entry points the
iteration goes through, averaged over N iterations (no profiler overhead).

    python scripts/kmeans_breakdown.py [--iters 200]
"""
import argparse
import collections
import functools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import core, engine  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402

T = collections.defaultdict(float)
N = collections.defaultdict(int)
_depth = [0]


def timed(mod, name, label=None):
    f = getattr(mod, name)

    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label or name] += time.perf_counter() - t0
            N[label or name] += 1
    setattr(mod, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    gpu = torch.cuda.is_available()
    dev = engine.compute_device()
    rng = np.random.default_rng(2)
    pts = rng.uniform(0.0, 1.0, size=(100_000 if gpu else 2_000, 100))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4))
    df = df.cache_on_device(dev) if gpu else df.cache()
    c = rng.standard_normal((10, 100))
    for _ in range(20):
        c, _ = kmeans.run_one_step2(df, c)
    for mod, name in [(core, "map_blocks"), (core, "reduce_blocks"), (core, "_resolve"), (core, "analyze_graph"),
                      (engine, "program"), (engine, "run_program"), (core, "_combine_monoids"),
                      (core, "_to_host_batched"), (engine, "cat_rows"), (kmeans, "tf_compute_distances")]:
        timed(mod, name)
    if gpu:
        torch.cuda.synchronize()
    T.clear()
    N.clear()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        c, _ = kmeans.run_one_step2(df, c)
    if gpu:
        torch.cuda.synchronize()
    total = (time.perf_counter() - t0) / a.iters * 1e6
    res = {"iteration_us": total,
           "us_per_iter": {k: v / a.iters * 1e6 for k, v in sorted(T.items(), key=lambda x: -x[1])},
           "calls_per_iter": {k: v / a.iters for k, v in N.items()}, "gpu": gpu}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()

"""Host time of the pieces of one K-Means iteration (run_one_step2, 100k x 100
f64, k = 10, 4 device-cached partitions): every timed function is wrapped
with perf_counter (exclusive of nested timed calls is NOT computed: the
numbers are inclusive), including the native Program methods.

    python scripts/kmeans_host_parts.py [--iters 300]
"""
import argparse
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
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402

T, N = {}, {}


def timed(name, fn):
    @functools.wraps(fn)
    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[name] = T.get(name, 0.0) + time.perf_counter() - t
            N[name] = N.get(name, 0) + 1
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    for mod, names in ((core, ["_resolve", "_map_blocks_frame", "_reduce_setup", "_dense_inputs", "_assemble",
                               "_combine_monoids", "_to_host_batched", "map_blocks", "reduce_blocks"]),
                       (engine, ["program_for_spec", "run_program", "cat_rows_many", "_tensor_of"])):
        for n in names:
            setattr(mod, n, timed(f"{mod.__name__.split('.')[-1]}.{n}", getattr(mod, n)))
    for n in ("rebind", "run"):
        try:
            setattr(_C.Program, n, timed(f"Program.{n}", getattr(_C.Program, n)))
        except (AttributeError, TypeError):
            pass
    gpu = torch.cuda.is_available()
    rng = np.random.default_rng(2)
    pts = rng.uniform(0.0, 1.0, size=(100_000 if gpu else 2_000, 100))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4))
    df = df.cache_on_device(engine.compute_device()) if gpu else df.cache()
    c = rng.standard_normal((10, 100))
    for _ in range(20):
        c, _ = kmeans.run_one_step2(df, c)
    T.clear()
    N.clear()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        c, _ = kmeans.run_one_step2(df, c)
    total = (time.perf_counter() - t0) / a.iters * 1e6
    print(json.dumps({"iteration_us": round(total, 1),
                      "inclusive_us_per_iter": {k: round(v / a.iters * 1e6, 1) for k, v in
                                                sorted(T.items(), key=lambda kv: -kv[1])},
                      "calls_per_iter": {k: round(v / a.iters, 2) for k, v in sorted(N.items())}}, indent=1))


if __name__ == "__main__":
    main()

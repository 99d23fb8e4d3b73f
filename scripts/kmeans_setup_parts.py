"""Host cost of the per-iteration graph setup of K-Means (run_one_step2's
map graph, 100 x 10 f64 centres changing every iteration): DSL build,
serialisation, content hash, native parse, structure key, graph rewrites,
Program construction and plan adoption, each timed on its own.

    python scripts/kmeans_setup_parts.py [--iters 300]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from tensorframes_amd import engine  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.graph import dsl as tf  # noqa: E402
from tensorframes_amd.models.kmeans import tf_compute_distances  # noqa: E402

T = {}


def lap(name, t0):
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


def one(c, old):
    t = time.perf_counter()
    with tf.Graph().as_default() as g:
        points = tf.placeholder(tf.double, shape=[None, 100], name="features")
        distances = tf_compute_distances(points, c)
        t = lap("dsl_distances", t)
        indexes = tf.argmin(distances, 1, name="indexes")
        min_distances = tf.reduce_min(distances, 1, name="min_distances")
        num_points = tf.stack([tf.shape(points)[0]], name="num_points")
        counts = tf.tile(tf.constant([1]), num_points, name="count")
        bp = tf.unsorted_segment_sum(points, indexes, 10, name="block_points")
        bc = tf.unsorted_segment_sum(counts, indexes, 10, name="block_counts")
        bd = tf.reduce_sum(min_distances, name="block_distances")
        tf.expand_dims(bp, 0, name="agg_points")
        tf.expand_dims(bc, 0, name="agg_counts")
        tf.expand_dims(bd, 0, name="agg_distances")
        t = lap("dsl_rest", t)
        b = g.serialize()
        t = lap("serialize", t)
    engine._key(b)
    t = lap("content_hash", t)
    ng = _C.Graph(b)
    t = lap("native_parse", t)
    sk = ng.structure_key()
    t = lap("structure_key", t)
    pb = engine._planned_bytes(b)
    t = lap("graph_rewrites", t)
    fetches = ["agg_counts:0", "agg_distances:0", "agg_points:0"]
    p = _C.Program(ng if pb is b else _C.Graph(pb), fetches, ["features"])
    t = lap("program_ctor", t)
    if old is not None:
        p.adopt(old)
    lap("adopt", t)
    return p, sk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    c = rng.standard_normal((10, 100))
    old = None
    for _ in range(20):
        c = c + 1e-3
        old, _ = one(c, old)
    T.clear()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        c = c + 1e-3
        old, _ = one(c, old)
    total = (time.perf_counter() - t0) / a.iters * 1e6
    print(json.dumps({"total_us": round(total, 1),
                      "parts_us": {k: round(v / a.iters * 1e6, 1) for k, v in T.items()}}, indent=1))


if __name__ == "__main__":
    main()

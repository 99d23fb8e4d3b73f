"""Phase timing of one K-Means iteration (run_one_step2 re-stated with
perf_counter checkpoints; 100k x 100 f64, k = 10, 4 device-cached
partitions): graph building (DSL), map_blocks (lazy setup), reduce graph
building, reduce_blocks (runs the map partitions + the reduce; ends in the
one device-to-host copy), and the numpy update of the centres.

    python scripts/kmeans_phases.py [--iters 200]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import core, engine  # noqa: E402
from tensorframes_amd.graph import dsl as tf  # noqa: E402
from tensorframes_amd.models.kmeans import tf_compute_distances  # noqa: E402

T = {}


def lap(name, t0):
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0)
    return t


def step(df, start_centers):
    t = time.perf_counter()
    num_centroids, num_features = np.shape(start_centers)
    with tf.Graph().as_default():
        points = tf.placeholder(tf.double, shape=[None, num_features], name="features")
        distances = tf_compute_distances(points, start_centers)
        indexes = tf.argmin(distances, 1, name="indexes")
        min_distances = tf.reduce_min(distances, 1, name="min_distances")
        num_points = tf.stack([tf.shape(points)[0]], name="num_points")
        counts = tf.tile(tf.constant([1]), num_points, name="count")
        block_points = tf.unsorted_segment_sum(points, indexes, num_centroids, name="block_points")
        block_counts = tf.unsorted_segment_sum(counts, indexes, num_centroids, name="block_counts")
        block_distances = tf.reduce_sum(min_distances, name="block_distances")
        agg_points = tf.expand_dims(block_points, 0, name="agg_points")
        agg_counts = tf.expand_dims(block_counts, 0, name="agg_counts")
        agg_distances = tf.expand_dims(block_distances, 0, name="agg_distances")
        t = lap("1_dsl_map_graph", t)
        df2 = core.map_blocks([agg_points, agg_counts, agg_distances], df, trim=True)
        t = lap("2_map_blocks_call", t)
    with tf.Graph().as_default():
        x_input = tf.placeholder(tf.double, shape=[None, num_centroids, num_features], name="agg_points_input")
        count_input = tf.placeholder(tf.int32, shape=[None, num_centroids], name="agg_counts_input")
        md_input = tf.placeholder(tf.double, shape=[None], name="agg_distances_input")
        x = tf.reduce_sum(x_input, [0], name="agg_points")
        count = tf.reduce_sum(count_input, [0], name="agg_counts")
        min_distances = tf.reduce_sum(md_input, [0], name="agg_distances")
        t = lap("3_dsl_reduce_graph", t)
        x_, count_, total = core.reduce_blocks([x, count, min_distances], df2)
        t = lap("4_reduce_blocks_call", t)
    new_centers = (x_.T / (count_ + 1e-7)).T
    lap("5_update", t)
    return new_centers, float(total)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    gpu = torch.cuda.is_available()
    rng = np.random.default_rng(2)
    pts = rng.uniform(0.0, 1.0, size=(100_000 if gpu else 2_000, 100))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4))
    df = df.cache_on_device(engine.compute_device()) if gpu else df.cache()
    c = rng.standard_normal((10, 100))
    for _ in range(20):
        c, _ = step(df, c)
    T.clear()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        c, _ = step(df, c)
    total = (time.perf_counter() - t0) / a.iters * 1e6
    print(json.dumps({"iteration_us": round(total, 1),
                      "phase_us": {k: round(v / a.iters * 1e6, 1) for k, v in sorted(T.items())}}, indent=1))


if __name__ == "__main__":
    main()

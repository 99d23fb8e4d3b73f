"""K-Means over a DataFrame of feature vectors, in the two styles of the
reference demo (reference: src/main/python/tensorframes_snippets/kmeans_demo.py:13-193):

* `run_one_step` — map_blocks computes each point's nearest centroid
  (MFMA f64 GEMM for the point/centroid products, arg-min), then
  `aggregate(groupBy(indexes))` sums the points per cluster (segmented
  reduction kernel);
* `run_one_step2` — everything inside one map_blocks(trim=True) per block
  (`UnsortedSegmentSum` pre-aggregation), then `reduce_blocks` sums the
  per-block partials (native reduction + RCCL all-reduce across GPUs).

The graphs are built with the TF-compatible DSL exactly as the reference
builds them with TensorFlow.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .. import core
from ..graph import dsl as tf


def tf_compute_distances(points, start_centers):
    """Squared distances [num_points, num_centroids] (reference: kmeans_demo.py:13-43)."""
    with tf.variable_scope("distances"):
        num_centroids, _ = np.shape(start_centers)
        num_points = tf.shape(points)[0]
        centers = tf.constant(start_centers)
        squares = tf.reduce_sum(tf.square(points), reduction_indices=1)
        center_squares = tf.reduce_sum(tf.square(centers), reduction_indices=1)
        prods = tf.matmul(points, centers, transpose_b=True)
        t1a = tf.expand_dims(center_squares, 0)
        t1b = tf.stack([num_points, 1])
        t1 = tf.tile(t1a, t1b)
        t2a = tf.expand_dims(squares, 1)
        t2b = tf.stack([1, num_centroids])
        t2 = tf.tile(t2a, t2b)
        distances = t1 + t2 - 2 * prods
    return distances


def run_one_step(dataframe, start_centers, features_col: str = "features") -> Tuple[np.ndarray, float]:
    """One iteration: map_blocks + groupBy/aggregate (reference: kmeans_demo.py:46-98)."""
    num_centroids, num_features = np.shape(start_centers)
    with tf.Graph().as_default():
        points = tf.placeholder(tf.double, shape=[None, num_features], name=features_col)
        num_points = tf.stack([tf.shape(points)[0]], name="num_points")
        distances = tf_compute_distances(points, start_centers)
        indexes = tf.argmin(distances, 1, name="indexes")
        min_distances = tf.reduce_min(distances, 1, name="min_distances")
        counts = tf.tile(tf.constant([1]), num_points, name="count")
        df2 = core.map_blocks([indexes, counts, min_distances], dataframe)
    gb = df2.groupBy("indexes")
    with tf.Graph().as_default():
        x_input = core.block(df2, features_col, tf_name=features_col + "_input")
        count_input = core.block(df2, "count", tf_name="count_input")
        md_input = core.block(df2, "min_distances", tf_name="min_distances_input")
        x = tf.reduce_sum(x_input, [0], name=features_col)
        count = tf.reduce_sum(count_input, [0], name="count")
        min_distances = tf.reduce_sum(md_input, [0], name="min_distances")
        df3 = core.aggregate([x, count, min_distances], gb)
    rows = df3.collect()
    new_centers = np.array(start_centers, dtype=np.float64).copy()
    for row in rows:
        new_centers[int(row.indexes)] = np.array(row[features_col]) / row["count"]
    total = float(np.sum([row["min_distances"] for row in rows]))
    return new_centers, total


def run_one_step2(dataframe, start_centers, features_col: str = "features") -> Tuple[np.ndarray, float]:
    """One iteration aggregated inside the graph (reference: kmeans_demo.py:101-168)."""
    num_centroids, num_features = np.shape(start_centers)
    with tf.Graph().as_default():
        points = tf.placeholder(tf.double, shape=[None, num_features], name=features_col)
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
        df2 = core.map_blocks([agg_points, agg_counts, agg_distances], dataframe, trim=True)
    with tf.Graph().as_default():
        x_input = tf.placeholder(tf.double, shape=[None, num_centroids, num_features], name="agg_points_input")
        count_input = tf.placeholder(tf.int32, shape=[None, num_centroids], name="agg_counts_input")
        md_input = tf.placeholder(tf.double, shape=[None], name="agg_distances_input")
        x = tf.reduce_sum(x_input, [0], name="agg_points")
        count = tf.reduce_sum(count_input, [0], name="agg_counts")
        min_distances = tf.reduce_sum(md_input, [0], name="agg_distances")
        x_, count_, total = core.reduce_blocks([x, count, min_distances], df2)
    new_centers = (x_.T / (count_ + 1e-7)).T
    return new_centers, float(total)


def kmeans(dataframe, init_centers, num_iters: int = 5, tf_aggregate: bool = True,
           features_col: str = "features") -> Tuple[np.ndarray, List[float]]:
    """Runs K-Means (reference: kmeans_demo.py:171-193)."""
    step = run_one_step2 if tf_aggregate else run_one_step
    c, d, ds = init_centers, np.inf, []
    for _ in range(num_iters):
        c1, d1 = step(dataframe, c, features_col)
        c = c1
        if d == d1:
            break
        d = d1
        ds.append(d1)
    return c, ds


def numpy_step(points: np.ndarray, centers: np.ndarray) -> Tuple[np.ndarray, float]:
    """Reference implementation of one Lloyd step (test oracle)."""
    d = (points ** 2).sum(1)[:, None] + (centers ** 2).sum(1)[None, :] - 2 * points @ centers.T
    idx = d.argmin(1)
    new = centers.copy()
    for k in range(centers.shape[0]):
        m = idx == k
        if m.any():
            new[k] = points[m].mean(0)
    return new, float(d.min(1).sum())

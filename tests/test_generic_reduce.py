"""Generic (non-monoid) reductions on the device: reduce_rows pair graphs are
lifted over a batch of row pairs (graph/vectorize.py) and folded as a tree,
log2(rows) launches per partition (reference:
DebugRowOps.scala:930-969 performReducePairwise, a sequential fold)."""
import time

import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.utils.logging import metrics


def _absmax_graph():
    a = tf.placeholder(tf.double, [3], name="x_1")
    b = tf.placeholder(tf.double, [3], name="x_2")
    return tf.maximum(tf.abs(a), tf.abs(b), name="x")  # associative, not a recognised monoid


@pytest.mark.parametrize("n,parts", [(1, 1), (2, 1), (3, 1), (7, 2), (1001, 3), (4096, 4)])
def test_tree_fold_matches_numpy(n, parts):
    x = np.random.default_rng(n).standard_normal((n, 3))
    df = tfs.from_columns({"x": x}, num_partitions=parts)
    before = metrics.snapshot().get("reduce_rows_tree_folds", 0)
    with tf.Graph().as_default():
        got = tfs.reduce_rows(_absmax_graph(), df)
    np.testing.assert_array_equal(got, np.abs(x).max(0))
    if n > 1:
        assert metrics.snapshot().get("reduce_rows_tree_folds", 0) > before


def test_tree_fold_two_columns_and_sequential_fallback_agree():
    rng = np.random.default_rng(3)
    x, y = rng.standard_normal((999, 2)), rng.integers(-5, 5, 999).astype(np.int64)
    df = tfs.from_columns({"x": x, "y": y}, num_partitions=3)

    def run():
        with tf.Graph().as_default():
            x1 = tf.placeholder(tf.double, [2], name="x_1")
            x2 = tf.placeholder(tf.double, [2], name="x_2")
            y1 = tf.placeholder(tf.int64, [], name="y_1")
            y2 = tf.placeholder(tf.int64, [], name="y_2")
            # x: hypot-style accumulate; y: sum of squares-free max(|.|)
            xo = tf.sqrt(x1 * x1 + x2 * x2, name="x")
            yo = tf.maximum(tf.abs(y1), tf.abs(y2), name="y")
            return tfs.reduce_rows([xo, yo], df)
    fast = run()
    tfs.set_config(map_rows_vectorize=False)
    try:
        slow = run()
    finally:
        tfs.set_config(map_rows_vectorize=True)
    np.testing.assert_allclose(fast[0], np.sqrt((x * x).sum(0)), rtol=1e-12)
    np.testing.assert_allclose(fast[0], slow[0], rtol=1e-12)
    assert fast[1] == slow[1] == np.abs(y).max()


def test_ragged_rows_keep_the_sequential_fold():
    rows = [tfs.Row(v=[1.0] * (1 + i % 3)) for i in range(6)]
    df = tfs.create_dataframe(rows, num_partitions=2)
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, [None], name="v_1")
        b = tf.placeholder(tf.double, [None], name="v_2")
        out = tf.identity(tf.reduce_sum(a, [0], keep_dims=True) + tf.reduce_sum(b, [0], keep_dims=True), name="v")
        got = tfs.reduce_rows(out, df)
    assert float(np.asarray(got).reshape(-1)[0]) == 12.0


def test_generic_reduce_rows_100k_rows_is_fast():
    """Round 2: 1.26 s per 100k rows through the per-row loop."""
    x = np.random.default_rng(4).standard_normal((100_000, 3))
    df = tfs.from_columns({"x": x}, num_partitions=4).cache()
    df.local_blocks()
    with tf.Graph().as_default():
        g = _absmax_graph()
        tfs.reduce_rows(g, df)
        t0 = time.perf_counter()
        got = tfs.reduce_rows(g, df)
        dt = time.perf_counter() - t0
    np.testing.assert_array_equal(got, np.abs(x).max(0))
    assert dt < 0.25, dt


@pytest.mark.gpu
def test_generic_reduce_rows_1m_rows_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    x = torch.randn((1_000_000, 3), dtype=torch.float64, device=dev)
    df = tfs.from_columns({"x": x}, num_partitions=4).cache_on_device(dev)
    with tf.Graph().as_default():
        g = _absmax_graph()
        tfs.reduce_rows(g, df)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = tfs.reduce_rows(g, df)
        dt = time.perf_counter() - t0
    np.testing.assert_array_equal(got, x.abs().max(0).values.cpu().numpy())
    print(f"generic reduce_rows 1M rows on the GPU: {dt * 1e3:.1f} ms")
    assert dt < 0.05, dt

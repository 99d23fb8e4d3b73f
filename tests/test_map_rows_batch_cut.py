"""map_rows batch-of-one cut (core._BatchCut): per-row preprocessing of
differently-shaped cells, then ONE run of the batch-1 model over a chunk of
rows. Results must equal the per-row loop; graphs that mix rows below the cut
must be refused (reference semantics: one session.run per row,
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:832-856)."""
import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.utils.logging import metrics

rng = np.random.default_rng(3)


def image_frame(n=7):
    imgs = [rng.uniform(0, 1, (int(rng.integers(6, 12)), int(rng.integers(6, 12)), 3)) for _ in range(n)]
    return tfs.analyze(tfs.create_dataframe([tfs.Row(img=[[list(p) for p in r] for r in im]) for im in imgs],
                                            num_partitions=2))


def scoring_graph(mix=None):
    w = rng.standard_normal((3, 3, 3, 4)).astype(np.float32)
    fc = rng.standard_normal((4 * 8 * 8, 10)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, None, 3], name="img")
        r = tf.image.resize_images(x, [8, 8])
        b = tf.expand_dims(r - 0.5, 0)
        y = tf.nn.relu(tf.nn.conv2d(b, tf.constant(w), [1, 1, 1, 1], "SAME"))
        if mix == "conv":  # mixes the batch-of-one: the cut moves below it
            y = y - tf.reduce_mean(y, [0], keep_dims=True)
        logits = tf.matmul(tf.reshape(y, [-1, 4 * 8 * 8]), tf.constant(fc))
        prob = tf.nn.softmax(logits, name="prob")
        sq = tf.squeeze(prob)
        if mix == "squeezed":  # a reduction over the squeezed row: no batched form
            sq = sq - tf.reduce_mean(sq)
        vals, idx = tf.nn.top_k(sq, 3, name="top")
        tf.identity(vals, name="value")
        tf.identity(idx, name="index")
    return g


def run_rows(g, df, vectorize):
    old = tfs.config.map_rows_vectorize
    tfs.set_config(map_rows_vectorize=vectorize)
    try:
        with g.as_default():
            out = tfs.map_rows([g.get_tensor_by_name("value:0"), g.get_tensor_by_name("index:0"),
                                g.get_tensor_by_name("prob:0")], df)
            return out.to_numpy("value"), out.to_numpy("index"), out.to_numpy("prob")
    finally:
        tfs.set_config(map_rows_vectorize=old)


def test_batch_cut_matches_per_row_loop():
    df = image_frame()
    g = scoring_graph()
    metrics.reset()
    v1, i1, p1 = run_rows(g, df, True)
    m = metrics.snapshot()  # (each to_numpy re-evaluates the lazy frame)
    assert m.get("map_rows_batch_cut_rows", 0) == m["map_rows_rows"] > 0
    v0, i0, p0 = run_rows(g, df, False)
    np.testing.assert_allclose(v1, v0, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(i1, i0)
    assert p1.shape == p0.shape == (7, 1, 10)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)


def test_cut_moves_below_a_batch_of_one_reduction():
    df = image_frame()
    g = scoring_graph(mix="conv")
    metrics.reset()
    v1, i1, _ = run_rows(g, df, True)
    m = metrics.snapshot()
    assert m.get("map_rows_batch_cut_rows", 0) == m["map_rows_rows"] > 0
    v0, i0, _ = run_rows(g, df, False)
    np.testing.assert_allclose(v1, v0, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(i1, i0)


def test_reduction_after_a_dropped_batch_dim_is_refused():
    df = image_frame()
    g = scoring_graph(mix="squeezed")
    metrics.reset()
    v1, _, _ = run_rows(g, df, True)
    assert metrics.snapshot().get("map_rows_batch_cut_rows", 0) == 0
    v0, _, _ = run_rows(g, df, False)
    np.testing.assert_allclose(v1, v0, rtol=1e-5, atol=1e-6)


def test_explicit_squeeze_dims():
    """squeeze(x, [0, 2]) keeps the batch dim and still drops dim 2."""
    df = image_frame(5)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, None, 3], name="img")
        r = tf.expand_dims(tf.image.resize_images(x, [4, 4]), 0)  # [1, 4, 4, 3]
        m = tf.reduce_max(r, [2], keep_dims=True)  # [1, 4, 1, 3]
        tf.identity(tf.nn.softmax(tf.squeeze(m, [0, 2])), name="value")  # [4, 3]
        tf.identity(m, name="index")
        tf.identity(r, name="prob")
    metrics.reset()
    v1, i1, _ = run_rows(g, df, True)
    m = metrics.snapshot()
    assert m.get("map_rows_batch_cut_rows", 0) == m["map_rows_rows"] > 0
    v0, i0, _ = run_rows(g, df, False)
    assert v1.shape == v0.shape == (5, 4, 3)
    np.testing.assert_allclose(v1, v0, rtol=1e-6)
    np.testing.assert_allclose(i1, i0, rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_batch_cut_on_gpu_matches_cpu_loop():
    """Rows forced onto the GPU: the per-row part runs on a side stream, the
    batched part on the compute stream; results equal the CPU per-row loop."""
    df = image_frame(150)  # > one chunk of 64 rows
    g = scoring_graph()
    old = tfs.config.map_rows_gpu_min_elems
    try:
        tfs.set_config(map_rows_gpu_min_elems=0)
        metrics.reset()
        v1, i1, p1 = run_rows(g, df, True)
        m = metrics.snapshot()
        assert m.get("map_rows_batch_cut_rows", 0) == m["map_rows_rows"] > 0
    finally:
        tfs.set_config(map_rows_gpu_min_elems=old)
    v0, i0, p0 = run_rows(g, df, False)
    np.testing.assert_allclose(p1, p0, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v1, v0, rtol=1e-4, atol=1e-5)


def test_batch_rows_config_chunks_the_rows():
    """7 rows in chunks of 3 (3 + 3 + 1): same results as the per-row loop."""
    df = image_frame()
    g = scoring_graph()
    old = tfs.config.map_rows_batch_rows
    try:
        tfs.set_config(map_rows_batch_rows=3)
        v1, i1, p1 = run_rows(g, df, True)
    finally:
        tfs.set_config(map_rows_batch_rows=old)
    v0, i0, p0 = run_rows(g, df, False)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(i1, i0)

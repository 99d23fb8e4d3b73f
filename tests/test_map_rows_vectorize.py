"""map_rows fast path: row graphs lifted to block graphs (graph/vectorize.py)
must give exactly the per-row results, and graphs that cannot be lifted must
fall back to the per-row loop."""
import numpy as np
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import Row, tf
from tensorframes_amd.utils.logging import metrics

rng = np.random.default_rng(5)
W = rng.standard_normal((4, 3))


def _frame(ragged=False):
    if ragged:
        rows = [Row(v=[float(x) for x in rng.standard_normal(2 + i % 3)], s=float(i)) for i in range(9)]
    else:
        rows = [Row(v=[float(x) for x in rng.standard_normal(4)], s=float(i)) for i in range(9)]
    return tfs.analyze(tfs.create_dataframe(rows, num_partitions=2))


def g_add(v, s):
    return tf.add(v, 3.0, name="o")


def g_mix(v, s):
    return tf.multiply(tf.square(v) + s, tf.constant([1.0, 2.0, 3.0, 4.0], dtype=tf.float64), name="o")


def g_reduce(v, s):
    return tf.add(tf.reduce_sum(v, [0]), tf.reduce_max(v, [-1]), name="o")


def g_argmax(v, s):
    return tf.identity(tf.argmax(v, 0), name="o")


def g_softmax(v, s):
    return tf.nn.softmax(tf.reshape(v, [2, 2]), name="o")


def g_expand_transpose(v, s):
    x = tf.expand_dims(v, 0)                      # [1, 4]
    y = tf.transpose(tf.concat([x, x * 2.0], 0))  # [4, 2]
    return tf.squeeze(tf.reduce_sum(tf.expand_dims(y, 0), [2], keep_dims=True), [0, 2], name="o")


def g_matmul(v, s):
    return tf.identity(tf.matmul(tf.reshape(v, [1, 4]), tf.constant(W)), name="o")


def g_pack_cast(v, s):
    return tf.cast(tf.stack([s, s * 2.0]) > 3.0, tf.int32, name="o")


def g_extra_ops(v, s):
    y = tf.pad(tf.nn.leaky_relu(v, 0.3), [[1, 2]], mode="REFLECT")
    a, b = tf.split(tf.cumsum(y, 0, reverse=True), [3, -1], 0)
    return tf.add(tf.reduce_sum(tf.clip_by_value(tf.reverse(b, [0]), -1.0, 1.0), [0]), tf.reduce_max(a, [0]),
                  name="o")


LIFTABLE = [g_add, g_mix, g_reduce, g_argmax, g_softmax, g_expand_transpose, g_matmul, g_pack_cast, g_extra_ops]


def _run(builder, df, vectorize):
    tfs.set_config(map_rows_vectorize=vectorize)
    try:
        with tf.Graph().as_default():
            v = tf.placeholder(tf.float64, [None], name="v")
            s = tf.placeholder(tf.float64, [], name="s")
            out = tfs.map_rows(builder(v, s), df)
            return [np.asarray(r.o) for r in out.collect()]
    finally:
        tfs.set_config(map_rows_vectorize=True)


@pytest.mark.parametrize("builder", LIFTABLE, ids=lambda f: f.__name__)
def test_lifted_graph_matches_per_row(builder):
    df = _frame()
    before = metrics.snapshot().get("map_rows_vectorized_rows", 0)
    fast = _run(builder, df, True)
    assert metrics.snapshot().get("map_rows_vectorized_rows", 0) - before == 9
    slow = _run(builder, df, False)
    for a, b in zip(fast, slow):
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)


def test_ragged_rows_group_by_shape():
    df = _frame(ragged=True)
    before = metrics.snapshot().get("map_rows_vectorized_rows", 0)
    fast = _run(g_reduce, df, True)
    assert metrics.snapshot().get("map_rows_vectorized_rows", 0) > before
    slow = _run(g_reduce, df, False)
    for a, b in zip(fast, slow):
        np.testing.assert_allclose(a, b, rtol=1e-12)


def _shape_dependent(v, s):
    return tf.cast(tf.shape(v), tf.float64) + s


def _const_outranks(v, s):
    return tf.add(s, tf.constant([1.0, 2.0], dtype=tf.float64), name="o")


@pytest.mark.parametrize("builder", [_shape_dependent, _const_outranks], ids=lambda f: f.__name__)
def test_unliftable_graphs_fall_back(builder):
    df = _frame()
    before = metrics.snapshot().get("map_rows_vectorized_rows", 0)
    with tf.Graph().as_default():
        v = tf.placeholder(tf.float64, [None], name="v")
        s = tf.placeholder(tf.float64, [], name="s")
        o = tf.identity(builder(v, s), name="out")
        got = [np.asarray(r.out) for r in tfs.map_rows(o, df).collect()]
    assert metrics.snapshot().get("map_rows_vectorized_rows", 0) == before
    assert len(got) == 9


def _matrix_frame(ms):
    rows = [Row(x=[[float(v) for v in rng.standard_normal(4)] for _ in range(m)]) for m in ms]
    return tfs.analyze(tfs.create_dataframe(rows, num_partitions=2))


def _matrix_rows(df):
    with tf.Graph().as_default():
        x = tf.placeholder(tf.float64, [None, 4], name="x")
        out = tfs.map_rows(tf.nn.relu(tf.matmul(x, tf.constant(W)), name="o"), df)
        return out.collect()


def test_lifted_matmul_keys_programs_by_cell_shape():
    # the lifted MatMul bakes the cell's row count m into a reshape: rows of
    # two different m in one call, and a second call with a third m, must each
    # get their own program (not the first one lifted for these ranks)
    for ms in ([2, 3] * 4, [5] * 4):
        df = _matrix_frame(ms)
        before = metrics.snapshot().get("map_rows_vectorized_rows", 0)
        got = _matrix_rows(df)
        assert metrics.snapshot().get("map_rows_vectorized_rows", 0) - before == len(ms)
        assert len(got) == len(ms)
        for r in got:
            x = np.asarray(r.x)
            np.testing.assert_allclose(np.asarray(r.o), np.maximum(x @ W, 0), rtol=1e-12, atol=1e-12)

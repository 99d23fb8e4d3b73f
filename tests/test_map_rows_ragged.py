"""map_rows over ragged cells: the whole-column grouped path (rows grouped by
cell shape with numpy, one lifted run per group, outputs assembled by index)
against a per-row numpy oracle. Reference behaviour: map_rows runs the row
graph once per row (src/main/scala/org/tensorframes/impl/DebugRowOps.scala:768-800)."""
import numpy as np

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.frame.block import RaggedColumn


def _frame(lens, seed=0):
    rng = np.random.default_rng(seed)
    rows = [(rng.standard_normal(int(n)).tolist(),) for n in lens]
    return tfs.analyze(tfs.create_dataframe(rows, ["v"])), [np.asarray(r[0]) for r in rows]


def test_ragged_scalar_output_matches_rows():
    lens = np.random.default_rng(1).integers(1, 9, 3000)
    df, cells = _frame(lens)
    with tf.Graph().as_default():
        v = tfs.row(df, "v")
        s = tf.reduce_sum(v * v, name="s")
        out = tfs.map_rows(s, df)
        got = np.array([r["s"] for r in out.collect()])
    want = np.array([(c * c).sum() for c in cells])
    np.testing.assert_allclose(got, want, rtol=1e-12)


def test_ragged_ragged_output_keeps_row_order():
    lens = np.random.default_rng(2).integers(1, 6, 2000)
    df, cells = _frame(lens, seed=3)
    with tf.Graph().as_default():
        v = tfs.row(df, "v")
        y = tf.add(v * 2.0, 1.0, name="y")
        out = tfs.map_rows(y, df)
        rows = out.collect()
    assert len(rows) == len(cells)
    for r, c in zip(rows, cells):
        np.testing.assert_allclose(np.asarray(r["y"]), c * 2.0 + 1.0, rtol=1e-12)


def test_ragged_singleton_group_falls_back():
    # one row has a unique length: the grouped path declines, rows still right
    lens = [3] * 50 + [7] + [2] * 40
    df, cells = _frame(lens, seed=4)
    with tf.Graph().as_default():
        v = tfs.row(df, "v")
        s = tf.reduce_max(v, name="m")
        got = np.array([r["m"] for r in tfs.map_rows(s, df).collect()])
    np.testing.assert_allclose(got, [c.max() for c in cells])


def test_grouped_columns_direct():
    """The grouped path assembles a RaggedColumn for ragged outputs."""
    from tensorframes_amd import core
    lens = [2, 3, 2, 3, 4, 4]
    df, cells = _frame(lens, seed=5)
    with tf.Graph().as_default():
        v = tfs.row(df, "v")
        y = tf.identity(v * 3.0, name="y")
        out = tfs.map_rows(y, df)
        blocks = out.local_blocks()
    col = [b.columns["y"] for b in blocks.values()]
    assert all(isinstance(c, RaggedColumn) or hasattr(c, "shape") for c in col)
    assert core is not None

"""Operator integration tests, ported from the reference's
src/test/scala/org/tensorframes/BasicOperationsSuite.scala (21 tests, f64
unless stated) and src/test/scala/org/tensorframes/TrimmingOperationsSuite.scala."""
import numpy as np
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import Row, tf
from tensorframes_amd.frame.types import IntegerType, StringType, StructField, StructType, DoubleType

import pytest as _pytest

# every test runs on the host executor and, gpu-marked, on the GPU (conftest.on_device)
pytestmark = _pytest.mark.usefixtures("on_device")


def make1(xs, col="x", num_partitions=1):
    return tfs.create_dataframe([(x,) for x in xs], [col], num_partitions=num_partitions)


def sorted_rows(rows):
    return sorted(rows, key=str)


def test_identity():
    df = make1([1.0, 2.0], "in")
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None], name="in")
        out = tf.identity(p, name="out")
        df2 = tfs.map_blocks(out, df)
    assert df2.collect() == [(1.0, 1.0), (2.0, 2.0)]


def test_simple_add():
    df = tfs.create_dataframe([(1.0, 1.1), (2.0, 2.2)], ["a", "b"])
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, shape=[None], name="a")
        b = tf.placeholder(tf.double, shape=[None], name="b")
        out = tf.add(a, b, name="out")
        rows = tfs.map_blocks(out, df).collect()
    np.testing.assert_allclose([r.out for r in rows], [2.1, 4.2])
    assert [r.a for r in rows] == [1.0, 2.0]


def test_identity_1_dim():
    df = tfs.analyze(tfs.create_dataframe([([1.0],), ([2.0],)], ["in"]))
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None, 1], name="in")
        df2 = tfs.map_blocks(tf.identity(p, name="out"), df)
    assert df2.collect() == [([1.0], [1.0]), ([2.0], [2.0])]


def test_simple_add_1_dim():
    df = tfs.analyze(tfs.create_dataframe([([1.0], [1.1]), ([2.0], [2.2])], ["a", "b"]))
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, shape=[None, 1], name="a")
        b = tf.placeholder(tf.double, shape=[None, 1], name="b")
        rows = tfs.map_blocks(tf.add(a, b, name="out"), df).collect()
    np.testing.assert_allclose([r.out for r in rows], [[2.1], [4.2]])


def test_reduce_sum_double():
    df = make1([1.0, 2.0])
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x2 = tf.placeholder(tf.double, shape=[], name="x_2")
        x = tf.add(x1, x2, name="x")
        assert tfs.reduce_rows(x, df) == 3.0


def test_reduce_sum_int():
    schema = StructType([StructField("x", IntegerType(), False)])
    df = tfs.create_dataframe([(1,), (2,), (3,), (4,)], schema)
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.int32, shape=[], name="x_1")
        x2 = tf.placeholder(tf.int32, shape=[], name="x_2")
        x = tf.add(x1, x2, name="x")
        assert tfs.reduce_rows(x, df) == 10


def test_map_rows_identity():
    df = make1([1.0, 2.0], "in")
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[], name="in")
        assert tfs.map_rows(tf.identity(p, name="out"), df).collect() == [(1.0, 1.0), (2.0, 2.0)]


def test_map_rows_add():
    df = tfs.create_dataframe([(1.0, 1.1), (2.0, 2.2)], ["a", "b"])
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, shape=[], name="a")
        b = tf.placeholder(tf.double, shape=[], name="b")
        rows = tfs.map_rows(tf.add(a, b, name="out"), df).collect()
    np.testing.assert_allclose([r.out for r in rows], [2.1, 4.2])


@pytest.mark.parametrize("cell", [[1], [None]])
def test_map_rows_identity_1_dim(cell):
    df = tfs.analyze(tfs.create_dataframe([([1.0],), ([2.0],)], ["in"]))
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=cell, name="in")
        assert tfs.map_rows(tf.identity(p, name="out"), df).collect() == [([1.0], [1.0]), ([2.0], [2.0])]


def test_map_rows_variable_sizes():
    df = tfs.create_dataframe([([1.0],), ([2.0, 2.1],)], ["in"])
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None], name="in")
        rows = tfs.map_rows(tf.identity(p, name="out"), df).collect()
    assert rows == [([1.0], [1.0]), ([2.0, 2.1], [2.0, 2.1])]


def test_map_rows_add_1_dim():
    df = tfs.analyze(tfs.create_dataframe([([1.0], [1.1]), ([2.0], [2.2])], ["a", "b"]))
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, shape=[1], name="a")
        b = tf.placeholder(tf.double, shape=[1], name="b")
        rows = tfs.map_rows(tf.add(a, b, name="out"), df).collect()
    np.testing.assert_allclose([r.out[0] for r in rows], [2.1, 4.2])


def test_map_rows_add_unknown_rows():
    df = tfs.create_dataframe([([1.0, 1.0], [1.1, 1.1]), ([2.0], [2.2])], ["a", "b"])
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, shape=[None], name="a")
        b = tf.placeholder(tf.double, shape=[None], name="b")
        rows = tfs.map_rows(tf.add(a, b, name="out"), df).collect()
    np.testing.assert_allclose(rows[0].out, [2.1, 2.1])
    np.testing.assert_allclose(rows[1].out, [4.2])


def _sum_graph(dtype=tf.double):
    xi = tf.placeholder(dtype, shape=[None], name="x_input")
    return tf.reduce_sum(xi, [0], name="x")


def test_reduce_block_sum_double():
    df = make1([1.0, 2.0])
    with tf.Graph().as_default():
        assert tfs.reduce_blocks(_sum_graph(), df) == 3.0


def test_reduce_block_with_extra_column():
    df = tfs.create_dataframe([("1", 1.0), ("2", 1.1), ("3", 2.0)], ["key2", "x"])
    with tf.Graph().as_default():
        assert tfs.reduce_blocks(_sum_graph(), df) == pytest.approx(4.1)


def test_reduce_block_fixed_block_size():
    df = tfs.analyze(make1([1.0, 2.0], num_partitions=2))
    assert tfs.explain(df).strip().endswith("double[1]")
    with tf.Graph().as_default():
        assert tfs.reduce_blocks(_sum_graph(), df) == 3.0


def test_aggregate_over_rows():
    schema = StructType([StructField("key", IntegerType(), False), StructField("x", DoubleType(), False)])
    df = tfs.create_dataframe([(1, 1.0), (1, 1.1), (2, 2.0)], schema)
    with tf.Graph().as_default():
        out = tfs.aggregate(_sum_graph(), df.groupBy("key"))
        rows = out.collect()
    assert [r.key for r in rows] == [1, 2]
    np.testing.assert_allclose([r.x for r in rows], [2.1, 2.0])
    assert out.columns == ["key", "x"]


@pytest.mark.parametrize("cell", [[[1.0]], [[1.0, 2.0]], [[1.0, 2.0], [3.0, 4.0]]])
def test_two_tensors(cell):
    df = tfs.analyze(tfs.create_dataframe([(cell,)], ["x"]))
    with tf.Graph().as_default():
        x = tfs.block(df, "x")
        rows = tfs.map_blocks(tf.identity(x, name="y"), df).collect()
    assert rows[0].y == cell


def test_two_tensors_output():
    schema = StructType([StructField("x", IntegerType(), False)])
    df = tfs.analyze(tfs.create_dataframe([(1,)], schema))
    with tf.Graph().as_default():
        y = tf.constant([[1.0]], dtype=tf.double, name="y")
        rows = tfs.map_rows(y, df).collect()
    assert rows[0].y == [[1.0]]


# --- trimming (reference: TrimmingOperationsSuite.scala:17-47)
@pytest.mark.parametrize("nrows,const,expect", [(2, [1.0], 1), (1, [1.0, 2.0], 2), (2, [1.0, 2.0], 2)])
def test_trim_constant_outputs(nrows, const, expect):
    df = make1([float(i) for i in range(nrows)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")  # noqa: F841 (input only)
        out = tf.constant(const, dtype=tf.double, name="out")
        df2 = tfs.map_blocks(out, df, trim=True)
        rows = df2.collect()
    assert df2.columns == ["out"]
    assert len(rows) == expect
    assert [r.out for r in rows] == const[:expect]


def test_trim_higher_rank():
    df = tfs.analyze(tfs.create_dataframe([([1.0],), ([2.0],)], ["x"]))
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None, 1], name="x")  # noqa: F841
        out = tf.constant([[1.0]], dtype=tf.double, name="out")
        rows = tfs.map_blocks(out, df, trim=True).collect()
    assert rows == [([1.0],)]


def test_trim_reduces_rows_and_drops_inputs():
    df = make1([1.0, 2.0, 3.0])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        s = tf.reshape(tf.reduce_sum(x), [1], name="s")
        rows = tfs.map_blocks(s, df, trim=True).collect()
    assert rows == [(6.0,)]


# --- validation errors (reference: DebugRowOps.scala:318-355)
def test_missing_column_error():
    df = make1([1.0])
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None], name="nope")
        with pytest.raises(ValueError, match="no column to match it"):
            tfs.map_blocks(tf.identity(p, name="z"), df)


def test_dtype_mismatch_error():
    df = make1([1.0])
    with tf.Graph().as_default():
        p = tf.placeholder(tf.float32, shape=[None], name="x")
        with pytest.raises(ValueError, match="not compatible with the data type"):
            tfs.map_blocks(tf.identity(p, name="z"), df)


def test_output_collision_error():
    df = tfs.create_dataframe([(1.0, 2.0)], ["x", "z"])
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None], name="x")
        with pytest.raises(ValueError, match="already exists"):
            tfs.map_blocks(tf.add(p, 1.0, name="z"), df)


def test_shape_mismatch_error():
    df = tfs.analyze(tfs.create_dataframe([([1.0, 2.0],)], ["x"]))
    with tf.Graph().as_default():
        p = tf.placeholder(tf.double, shape=[None, 3], name="x")
        with pytest.raises(ValueError, match="not compatible"):
            tfs.map_blocks(tf.identity(p, name="z"), df)


def test_append_mode_row_count_error():
    df = make1([1.0, 2.0])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        s = tf.reshape(tf.reduce_sum(x), [1], name="s")
        with pytest.raises(ValueError, match="keep the number of rows"):
            tfs.map_blocks(s, df).collect()


def test_reduce_rows_must_cover_all_columns():
    df = tfs.create_dataframe([(1.0, 2.0)], ["x", "y"])
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x2 = tf.placeholder(tf.double, shape=[], name="x_2")
        with pytest.raises(ValueError, match="outputs are missing"):
            tfs.reduce_rows(tf.add(x1, x2, name="x"), df)


def test_reduce_blocks_extra_input_error():
    df = make1([1.0])
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        extra = tf.placeholder(tf.double, shape=[None], name="other")
        with pytest.raises(ValueError, match="Extra graph inputs"):
            tfs.reduce_blocks(tf.reduce_sum(xi + extra, [0], name="x"), df)


def test_reduce_empty_dataframe_error():
    df = tfs.create_dataframe([], StructType([StructField("x", DoubleType(), False)]))
    with tf.Graph().as_default():
        with pytest.raises(ValueError, match="empty"):
            tfs.reduce_blocks(_sum_graph(), df)


def test_null_values_rejected():
    with pytest.raises(ValueError, match="null"):
        tfs.create_dataframe([(1.0,), (None,)], ["x"])


def test_lazy_evaluation():
    calls = []
    df = make1([1.0, 2.0])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        df2 = tfs.map_blocks(tf.add(x, 1.0, name="z"), df)
    from tensorframes_amd.utils.logging import metrics
    before = metrics.snapshot().get("map_blocks_rows", 0)
    assert metrics.snapshot().get("map_blocks_rows", 0) == before  # nothing ran yet
    assert df2.count() == 2
    assert metrics.snapshot().get("map_blocks_rows", 0) == before + 2


def test_multiple_partitions_and_empty_partitions():
    df = make1([1.0, 2.0, 3.0], num_partitions=5)  # some partitions are empty
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        rows = tfs.map_blocks(tf.multiply(x, 2.0, name="z"), df).collect()
    with tf.Graph().as_default():
        assert tfs.reduce_blocks(_sum_graph(), df) == 6.0
    assert [r.z for r in rows] == [2.0, 4.0, 6.0]


def test_feed_dict_map_blocks_extension():
    df = make1([1.0, 2.0], "y")
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        rows = tfs.map_blocks(tf.add(x, 3.0, name="z"), df, feed_dict={"x": "y"}).collect()
    assert [r.z for r in rows] == [4.0, 5.0]


def test_graphdef_bytes_and_string_fetches():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        tf.add(x, 3.0, name="z")
    df = make1([1.0])
    rows = tfs.map_blocks("z", df, graph=g.serialize()).collect()
    assert rows == [(4.0, 1.0)]
    rows = tfs.map_blocks(["z:0"], df, graph=g.as_graph_def()).collect()
    assert rows == [(4.0, 1.0)]

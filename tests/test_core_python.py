"""Port of the reference's Python integration tests
(reference: src/main/python/tensorframes/core_test.py:34-127), with the
TensorFlow import replaced by `tensorframes_amd.tf` and Spark by our frame.
`test_reduce_blocks_1` is marked "This test fails" upstream; it passes here."""
import tensorframes_amd as tfs
from tensorframes_amd import Row, tf

import pytest as _pytest

# every test runs on the host executor and, gpu-marked, on the GPU (conftest.on_device)
pytestmark = _pytest.mark.usefixtures("on_device")


def test_schema(capsys):
    data = [Row(x=float(x)) for x in range(100)]
    df = tfs.create_dataframe(data)
    tfs.print_schema(df)
    assert "x: double" in capsys.readouterr().out


def test_map_blocks_1():
    df = tfs.create_dataframe([Row(x=float(x)) for x in range(10)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")
        df2 = tfs.map_blocks(z, df)
    data2 = df2.collect()
    assert data2[0].z == 3.0, data2


def test_map_rows_1():
    df = tfs.create_dataframe([Row(x=float(x)) for x in range(5)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[], name="x")
        z = tf.add(x, 3, name="z")
        df2 = tfs.map_rows(z, df)
    data2 = df2.collect()
    assert data2[0].z == 3.0, data2


def test_map_rows_2():
    df = tfs.create_dataframe([Row(y=float(y)) for y in range(5)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[], name="x")
        z = tf.add(x, 3, name="z")
        df2 = tfs.map_rows(z, df, feed_dict={"x": "y"})
    data2 = df2.collect()
    assert data2[0].z == 3.0, data2


def test_reduce_rows_1():
    data = [Row(x=float(x)) for x in range(5)]
    df = tfs.create_dataframe(data)
    with tf.Graph().as_default():
        x_1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x_2 = tf.placeholder(tf.double, shape=[], name="x_2")
        x = tf.add(x_1, x_2, name="x")
        res = tfs.reduce_rows(x, df)
    assert res == sum([r.x for r in data])


def test_reduce_blocks_1():
    data = [Row(x=float(x)) for x in range(5)]
    df = tfs.create_dataframe(data)
    with tf.Graph().as_default():
        x_input = tf.placeholder(tf.double, shape=[None], name="x_input")
        x = tf.reduce_sum(x_input, name="x")
        res = tfs.reduce_blocks(x, df)
    assert res == sum([r.x for r in data])


def test_map_blocks_trimmed_1():
    df = tfs.create_dataframe([Row(x=float(x)) for x in range(3)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")  # noqa: F841
        z = tf.constant([2], name="z")
        df2 = tfs.map_blocks(z, df, trim=True)
    data2 = df2.collect()
    assert data2[0].z == 2, data2


def test_groupby_1():
    data = [Row(x=float(x), key=str(x % 2)) for x in range(4)]
    df = tfs.create_dataframe(data)
    gb = df.groupBy("key")
    with tf.Graph().as_default():
        x_input = tfs.block(df, "x", tf_name="x_input")
        x = tf.reduce_sum(x_input, [0], name="x")
        df2 = tfs.aggregate(x, gb)
    data2 = df2.collect()
    assert data2 == [Row(key="0", x=2.0), Row(key="1", x=4.0)], data2


def test_multiple_fetches_return_list():
    df = tfs.create_dataframe([Row(x=float(x), y=float(2 * x)) for x in range(4)])
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        yi = tf.placeholder(tf.double, shape=[None], name="y_input")
        x = tf.reduce_sum(xi, [0], name="x")
        y = tf.reduce_min(yi, [0], name="y")
        res = tfs.reduce_blocks([x, y], df)
    assert res == [6.0, 0.0]


def test_vector_reduce_returns_numpy():
    import numpy as np
    df = tfs.analyze(tfs.create_dataframe([Row(x=[1.0, 2.0]), Row(x=[3.0, 4.0])]))
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None, 2], name="x_input")
        res = tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df)
    assert isinstance(res, np.ndarray)
    assert res.tolist() == [4.0, 6.0]

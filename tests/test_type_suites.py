"""Type-generic identity + monoid tests, instantiated for Int, Long, Float and
Double like the reference's src/test/scala/org/tensorframes/type_suites.scala:8-213
(tests written once, values converted per type)."""
import numpy as np
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.frame.types import (ArrayType, DoubleType, FloatType, IntegerType, LongType,
                                          StringType, StructField, StructType)

import pytest as _pytest

# every test runs on the host executor and, gpu-marked, on the GPU (conftest.on_device)
pytestmark = _pytest.mark.usefixtures("on_device")

TYPES = [
    (IntegerType(), tf.int32, int),
    (LongType(), tf.int64, int),
    (FloatType(), tf.float32, float),
    (DoubleType(), tf.float64, float),
]


@pytest.fixture(params=TYPES, ids=["int", "long", "float", "double"])
def T(request):
    return request.param


def df1(T, values, col="x", nested=False, analyzed=False, num_partitions=1):
    sql, _, py = T
    dt = ArrayType(sql, False) if nested else sql
    conv = (lambda v: [py(u) for u in v]) if nested else py
    df = tfs.create_dataframe([(conv(v),) for v in values], StructType([StructField(col, dt, False)]),
                              num_partitions=num_partitions)
    return tfs.analyze(df) if analyzed else df


# ---- identity tests (type_suites.scala:11-66)
def test_map_blocks_identity(T):
    df = df1(T, [1, 2])
    with tf.Graph().as_default():
        p = tf.placeholder(T[1], shape=[None], name="x")
        assert tfs.map_blocks(tf.identity(p, name="y"), df).collect() == [(1, 1), (2, 2)]


def test_map_blocks_identity_1d(T):
    df = df1(T, [[1], [2]], nested=True, analyzed=True)
    with tf.Graph().as_default():
        p = tf.placeholder(T[1], shape=[None, 1], name="x")
        assert tfs.map_blocks(tf.identity(p, name="y"), df).collect() == [([1], [1]), ([2], [2])]


@pytest.mark.parametrize("cell", [[1], [None]])
def test_map_rows_identity_1d(T, cell):
    df = df1(T, [[1], [2]], nested=True, analyzed=True)
    with tf.Graph().as_default():
        p = tf.placeholder(T[1], shape=cell, name="x")
        assert tfs.map_rows(tf.identity(p, name="y"), df).collect() == [([1], [1]), ([2], [2])]


def test_map_rows_identity_ragged(T):
    df = df1(T, [[1], [2, 3]], nested=True)
    with tf.Graph().as_default():
        p = tf.placeholder(T[1], shape=[None], name="x")
        assert tfs.map_rows(tf.identity(p, name="y"), df).collect() == [([1], [1]), ([2, 3], [2, 3])]


# ---- monoid tests (type_suites.scala:74-186)
def test_map_blocks_add(T):
    df = tfs.create_dataframe([(T[2](1), T[2](2))], StructType([StructField("a", T[0], False),
                                                               StructField("b", T[0], False)]))
    with tf.Graph().as_default():
        a = tf.placeholder(T[1], shape=[None], name="a")
        b = tf.placeholder(T[1], shape=[None], name="b")
        assert tfs.map_blocks(tf.add(a, b, name="c"), df).collect() == [(3, 1, 2)]


def test_map_blocks_add_1d(T):
    sql = ArrayType(T[0], False)
    df = tfs.analyze(tfs.create_dataframe([([T[2](1)], [T[2](2)])],
                                          StructType([StructField("a", sql, False), StructField("b", sql, False)])))
    with tf.Graph().as_default():
        a = tf.placeholder(T[1], shape=[None, 1], name="a")
        b = tf.placeholder(T[1], shape=[None, 1], name="b")
        assert tfs.map_blocks(tf.add(a, b, name="c"), df).collect() == [([3], [1], [2])]


def test_reduce_rows_sum(T):
    df = df1(T, [1, 2])
    with tf.Graph().as_default():
        x1 = tf.placeholder(T[1], shape=[], name="x_1")
        x2 = tf.placeholder(T[1], shape=[], name="x_2")
        assert tfs.reduce_rows(tf.add(x1, x2, name="x"), df) == 3


def test_reduce_rows_generic_graph(T):
    # not a recognised monoid form -> sequential fold path
    df = df1(T, [1, 2, 3], num_partitions=2)
    with tf.Graph().as_default():
        x1 = tf.placeholder(T[1], shape=[], name="x_1")
        x2 = tf.placeholder(T[1], shape=[], name="x_2")
        x = tf.identity(tf.add(x1, x2), name="x")
        assert tfs.reduce_rows(x, df) == 6


def test_map_rows_identity(T):
    df = df1(T, [1, 2])
    with tf.Graph().as_default():
        p = tf.placeholder(T[1], shape=[], name="x")
        assert tfs.map_rows(tf.identity(p, name="y"), df).collect() == [(1, 1), (2, 2)]


def test_map_rows_add(T):
    df = tfs.create_dataframe([(T[2](1), T[2](2))], StructType([StructField("a", T[0], False),
                                                               StructField("b", T[0], False)]))
    with tf.Graph().as_default():
        a = tf.placeholder(T[1], shape=[], name="a")
        b = tf.placeholder(T[1], shape=[], name="b")
        assert tfs.map_rows(tf.add(a, b, name="c"), df).collect() == [(3, 1, 2)]


def test_map_rows_add_1d_and_ragged(T):
    sql = ArrayType(T[0], False)
    schema = StructType([StructField("a", sql, False), StructField("b", sql, False)])
    df = tfs.create_dataframe([([T[2](1)], [T[2](2)]), ([T[2](1), T[2](1)], [T[2](2), T[2](3)])], schema)
    with tf.Graph().as_default():
        a = tf.placeholder(T[1], shape=[None], name="a")
        b = tf.placeholder(T[1], shape=[None], name="b")
        rows = tfs.map_rows(tf.add(a, b, name="c"), df).collect()
    assert [r.c for r in rows] == [[3], [3, 4]]


def test_reduce_blocks_sum(T):
    df = df1(T, [1, 2])
    with tf.Graph().as_default():
        xi = tf.placeholder(T[1], shape=[None], name="x_input")
        assert tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df) == 3


def test_reduce_blocks_with_string_column(T):
    schema = StructType([StructField("s", StringType(), False), StructField("x", T[0], False)])
    df = tfs.create_dataframe([("a", T[2](20)), ("b", T[2](21))], schema)
    with tf.Graph().as_default():
        xi = tf.placeholder(T[1], shape=[None], name="x_input")
        assert tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df) == 41


def test_aggregate(T):
    schema = StructType([StructField("key", StringType(), False), StructField("x", T[0], False)])
    df = tfs.create_dataframe([("a", T[2](10)), ("a", T[2](11)), ("b", T[2](20))], schema)
    with tf.Graph().as_default():
        xi = tf.placeholder(T[1], shape=[None], name="x_input")
        rows = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("key")).collect()
    assert rows == [("a", 21), ("b", 20)]


def test_reduce_min_and_max(T):
    df = df1(T, [5, 2, 9, 4], num_partitions=3)
    with tf.Graph().as_default():
        xi = tf.placeholder(T[1], shape=[None], name="x_input")
        assert tfs.reduce_blocks(tf.reduce_min(xi, [0], name="x"), df) == 2
    with tf.Graph().as_default():
        xi = tf.placeholder(T[1], shape=[None], name="x_input")
        assert tfs.reduce_blocks(tf.reduce_max(xi, [0], name="x"), df) == 9

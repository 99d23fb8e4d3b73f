"""PySpark interop (frame/spark_io.py) with stand-in Spark objects: pyspark is
not installed here, so the tests use duck-typed fakes that expose the pyspark
surface the adapter touches (DataFrame.toArrow / schema / rdd / limit,
GroupedData._df / _jgd, SparkSession.createDataFrame, pyspark.sql.types).
The operators are the reference's (src/main/python/tensorframes/core.py), called
with a "Spark" DataFrame as the reference's users do."""
import json
import sys
import types

import numpy as np
import pyarrow as pa
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.frame import spark_io

SHAPE_KEY, TYPE_KEY = "org.spartf.shape", "org.sparktf.type"


class _Field:
    def __init__(self, name, metadata=None):
        self.name, self.metadata = name, metadata or {}


class _Schema:
    def __init__(self, fields):
        self.fields = fields


class _RDD:
    def __init__(self, n):
        self._n = n

    def getNumPartitions(self):  # noqa: N802
        return self._n


class FakeSparkDF:
    def __init__(self, table, meta=None, parts=2):
        self._t, self._meta, self._parts = table, meta or {}, parts
        self.schema = _Schema([_Field(n, self._meta.get(n)) for n in table.column_names])
        self.rdd = _RDD(parts)

    def toArrow(self):  # noqa: N802
        return self._t

    def limit(self, n):
        return FakeSparkDF(self._t.slice(0, n), self._meta, 1)


FakeSparkDF.__module__ = "pyspark.sql.dataframe"


class _Expr:
    def __init__(self, s):
        self._s = s

    def sql(self):
        return f"`{self._s}`"


class _It:
    def __init__(self, xs):
        self._xs = list(xs)

    def hasNext(self):  # noqa: N802
        return bool(self._xs)

    def next(self):
        return self._xs.pop(0)


class _Seq:
    def __init__(self, xs):
        self._xs = xs

    def iterator(self):
        return _It(self._xs)


class _JGD:
    def __init__(self, keys):
        self._keys = keys

    def groupingExprs(self):  # noqa: N802
        return _Seq([_Expr(k) for k in self._keys])


class GroupedData:
    def __init__(self, df, keys):
        self._df, self._jgd = df, _JGD(keys)


GroupedData.__module__ = "pyspark.sql.group"


def vec_df():
    y = np.arange(20, dtype=np.float64).reshape(10, 2)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(y.reshape(-1)), 2)
    t = pa.table({"y": arr, "k": pa.array([i % 2 for i in range(10)], pa.int32())})
    meta = {"y": {SHAPE_KEY: [-1, 2], TYPE_KEY: "DoubleType"}}
    return FakeSparkDF(t, meta), y


def test_detection():
    sdf, _ = vec_df()
    assert spark_io.is_spark_dataframe(sdf)
    assert not spark_io.is_spark_dataframe(tfs.create_dataframe([tfs.Row(x=1.0)]))
    assert spark_io.is_spark_grouped(GroupedData(sdf, ["k"]))


def test_from_spark_keeps_metadata_and_partitions():
    sdf, y = vec_df()
    df = tfs.from_spark(sdf)
    assert df.num_partitions == 2
    assert df.schema["y"].metadata[SHAPE_KEY] == [-1, 2]
    np.testing.assert_array_equal(df.to_numpy("y"), y)


def test_operators_accept_spark_dataframes():
    sdf, y = vec_df()
    with tf.Graph().as_default():
        yb = tfs.block(sdf, "y")  # placeholder shape from the Spark field metadata
        assert yb.get_shape().as_list() == [None, 2]
        z = tf.add(yb, 3.0, name="z")
        out = tfs.map_blocks(z, sdf)
    np.testing.assert_allclose(out.to_numpy("z"), y + 3)
    with tf.Graph().as_default():
        yi = tf.placeholder(tf.float64, [None, 2], name="y_input")
        s = tfs.reduce_blocks(tf.reduce_sum(yi, [0], name="y"), sdf)
    np.testing.assert_allclose(s, y.sum(0))


def test_aggregate_accepts_spark_grouped_data():
    sdf, y = vec_df()
    with tf.Graph().as_default():
        yi = tf.placeholder(tf.float64, [None, 2], name="y_input")
        res = tfs.aggregate(tf.reduce_sum(yi, [0], name="y"), GroupedData(sdf, ["k"]))
    got = {r.k: np.asarray(r.y) for r in res.collect()}
    np.testing.assert_allclose(got[0], y[0::2].sum(0))
    np.testing.assert_allclose(got[1], y[1::2].sum(0))


def test_print_schema_of_spark_dataframe(capsys):
    sdf, _ = vec_df()
    tfs.print_schema(sdf)
    assert "double[?,2]" in capsys.readouterr().out


@pytest.fixture
def fake_pyspark(monkeypatch):
    """Minimal pyspark.sql.types so that to_spark's schema mapping runs."""
    T = types.ModuleType("pyspark.sql.types")

    class _T:
        def __init__(self, *a, **k):
            self.args, self.kw = a, k

        def __repr__(self):
            return f"{type(self).__name__}{self.args}"
    for n in ["DoubleType", "FloatType", "IntegerType", "LongType", "BooleanType", "StringType", "BinaryType",
              "ArrayType", "StructType", "StructField"]:
        setattr(T, n, type(n, (_T,), {}))
    sql = types.ModuleType("pyspark.sql")
    sql.types = T
    pyspark = types.ModuleType("pyspark")
    pyspark.sql = sql
    monkeypatch.setitem(sys.modules, "pyspark", pyspark)
    monkeypatch.setitem(sys.modules, "pyspark.sql", sql)
    monkeypatch.setitem(sys.modules, "pyspark.sql.types", T)
    return T


def test_to_spark_schema_and_rows(fake_pyspark):
    df = tfs.analyze(tfs.create_dataframe([tfs.Row(x=float(i), v=[1.0 * i, 2.0 * i]) for i in range(4)]))

    class Session:
        def createDataFrame(self, pdf, schema=None):  # noqa: N802
            self.pdf, self.schema = pdf, schema
            return "spark-df"
    sess = Session()
    assert tfs.to_spark(df, sess) == "spark-df"
    fields = {f.args[0]: f for f in sess.schema.args[0]}
    assert type(fields["x"].args[1]).__name__ == "DoubleType"
    arr = fields["v"].args[1]
    assert type(arr).__name__ == "ArrayType" and type(arr.args[0]).__name__ == "DoubleType"
    assert fields["v"].args[3][SHAPE_KEY] == [4, 2]
    assert sess.pdf["v"].iloc[3] == [3.0, 6.0]
    json.dumps(fields["v"].args[3])  # metadata stays JSON-serialisable for Spark

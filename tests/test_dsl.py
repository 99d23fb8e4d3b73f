"""DSL tests: NodeDefs must match TF-1.x text protos (golden), naming rules,
shape inference, and DSL graphs executing through the operators
(reference: src/test/scala/org/tensorframes/dsl/BasicSuite.scala:12-33,
dsl/BasicOpsSuite.scala:12-22, DSLOperationsSuite.scala:13-70,
TFInitializationSuite.scala:12-34)."""
import numpy as np
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.graph import proto as P


def texts(g):
    return {n.name: P.node_to_text(n) for n in g.as_graph_def().node}


CONST3 = '''name: "Const"
op: "Const"
attr {
  key: "dtype"
  value {
    type: DT_INT32
  }
}
attr {
  key: "value"
  value {
    tensor {
      dtype: DT_INT32
      tensor_shape {
      }
      int_val: 3
    }
  }
}
'''


def test_golden_constant():
    g = tf.Graph()
    with g.as_default():
        tf.constant(3)
    assert texts(g)["Const"] == CONST3


def test_golden_named_constant():
    g = tf.Graph()
    with g.as_default():
        tf.constant(3, name="x")
    assert texts(g)["x"] == CONST3.replace('name: "Const"', 'name: "x"')


def test_two_constants_same_name():
    g = tf.Graph()
    with g.as_default():
        a = tf.constant(3)
        b = tf.constant(3)
    assert (a.op.name, b.op.name) == ("Const", "Const_1")


def test_golden_fill():
    g = tf.Graph()
    with g.as_default():
        tf.fill([2], 3)
    t = texts(g)
    assert set(t) == {"Fill", "Fill/dims", "Fill/value"}
    assert t["Fill"] == '''name: "Fill"
op: "Fill"
input: "Fill/dims"
input: "Fill/value"
attr {
  key: "T"
  value {
    type: DT_INT32
  }
}
'''
    assert "int_val: 2" in t["Fill/dims"] and "size: 1" in t["Fill/dims"]
    assert "int_val: 3" in t["Fill/value"]


def test_golden_add():
    g = tf.Graph()
    with g.as_default():
        x = tf.constant(1, name="x")
        y = tf.constant(2, name="y")
        tf.add(x, y, name="z")
    assert texts(g)["z"] == '''name: "z"
op: "Add"
input: "x"
input: "y"
attr {
  key: "T"
  value {
    type: DT_INT32
  }
}
'''


def test_golden_placeholder_and_reduce():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x_input")
        tf.reduce_sum(x, [0], name="x")
    t = texts(g)
    assert t["x_input"] == '''name: "x_input"
op: "Placeholder"
attr {
  key: "dtype"
  value {
    type: DT_DOUBLE
  }
}
attr {
  key: "shape"
  value {
    shape {
      dim {
        size: -1
      }
    }
  }
}
'''
    assert 'input: "x/reduction_indices"' in t["x"]
    assert 'key: "keep_dims"' in t["x"] and 'key: "Tidx"' in t["x"]


def test_scalar_lifting_names_and_dtype():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")
        w = 3.0 + x
    assert z.op.inputs[1].op.name == "z/y"
    assert z.op.inputs[1].dtype == tf.double
    assert w.op.name == "add"


def test_name_scopes():
    g = tf.Graph()
    with g.as_default():
        with tf.name_scope("a"):
            c = tf.constant(1.0)
            with tf.name_scope("b"):
                d = tf.constant(2.0, name="d")
        with tf.name_scope("a"):
            e = tf.constant(3.0)
    assert (c.op.name, d.op.name, e.op.name) == ("a/Const", "a/b/d", "a_1/Const")


def test_graphs_are_isolated_per_context():
    with tf.Graph().as_default():
        a = tf.constant(1)
    with tf.Graph().as_default():
        b = tf.constant(1)
    assert a.op.name == b.op.name == "Const"


def test_shape_inference():
    with tf.Graph().as_default():
        x = tf.placeholder(tf.float32, shape=[None, 3], name="x")
        m = tf.matmul(x, tf.constant(np.ones((3, 5), np.float32)))
        assert m.get_shape().as_list() == [None, 5]
        s = tf.reduce_sum(m, [0])
        assert s.get_shape().as_list() == [5]
        s2 = tf.reduce_sum(m)
        assert s2.get_shape().as_list() == []
        b = tf.constant([[1.0], [2.0]]) + tf.constant([1.0, 2.0, 3.0])
        assert b.get_shape().as_list() == [2, 3]
        r = tf.reshape(x, [-1])
        assert r.get_shape().as_list() == [None]
        c = tf.nn.conv2d(tf.placeholder(tf.float32, [None, 299, 299, 3]), tf.constant(np.zeros((3, 3, 3, 32), np.float32)),
                         [1, 2, 2, 1], "VALID")
        assert c.get_shape().as_list() == [None, 149, 149, 32]
        sl = tf.shape(x)[0]
        assert sl.get_shape().as_list() == []


def test_session_run():
    with tf.Graph().as_default() as g:
        x = tf.placeholder(tf.float64, shape=[None], name="x")
        y = tf.reduce_sum(x * x, name="y")
        with tf.Session(device="cpu") as s:
            assert s.run(y, {x: np.array([1.0, 2.0, 3.0])}) == 14.0


# --- DSLOperationsSuite
def test_dsl_reduce_map_rows():
    df = tfs.create_dataframe([(1,)], ["a"])
    with tf.Graph().as_default():
        x = tf.constant([1.0, 1.0], dtype=tf.double, name="x")
        out = tf.reduce_sum(x, [0], name="out")
        assert out.get_shape().as_list() == []
        df2 = tfs.map_rows(out, df).select("a", "out")
    assert df2.collect() == [tfs.Row(a=1, out=2.0)]


def test_dsl_constant_map_rows():
    df = tfs.create_dataframe([(1,)], ["a"])
    with tf.Graph().as_default():
        x = tf.constant(1.0, dtype=tf.double, name="x")
        df2 = tfs.map_rows(x, df).select("a", "x")
    assert df2.collect() == [tfs.Row(a=1, x=1.0)]


def test_dsl_map_multiple_outputs():
    df = tfs.create_dataframe([(1.0,), (2.0,)], ["x"])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        y = tf.identity(x, name="y")
        z = tf.add(x, x, name="z")
        df2 = tfs.map_blocks([y, z], df).select("x", "y", "z")
    assert df2.collect() == [(1.0, 1.0, 2.0), (2.0, 2.0, 4.0)]


def test_dsl_row_and_block_extraction():
    df = tfs.create_dataframe([(1.0,), (2.0,)], ["a"])
    with tf.Graph().as_default():
        a = df.row("a")
        assert a.get_shape().as_list() == []
        b = tf.add(a, 2.0, name="b")
        rows = tfs.map_rows(b, df).select("a", "b").collect()
    assert rows == [(1.0, 3.0), (2.0, 4.0)]
    with tf.Graph().as_default():
        a = df.block("a")
        b = tf.add(a, 2.0, name="b")
        rows = df.map_blocks(b).select("a", "b").collect()
    assert rows == [(1.0, 3.0), (2.0, 4.0)]


def test_analyze_graph_summary():
    """TFInitializationSuite: graph analysis of DSL graphs."""
    with tf.Graph().as_default() as g:
        x = tf.placeholder(tf.double, shape=[None, 2], name="x")
        y = tf.add(x, x, name="y")
    from tensorframes_amd.core import _resolve, analyze_graph
    s = analyze_graph(_resolve(y))
    assert s["x"].is_input and s["x"].is_placeholder and not s["x"].is_output
    assert s["y"].is_output and not s["y"].is_input
    assert str(s["y"].shape) == "[?,2]"
    from tensorframes_amd.utils import dtypes as D
    assert s["y"].tf_dtype == D.DT_DOUBLE


def test_static_rank_matches_inference_and_skips_it():
    """reduce_*(x) over all axes takes x's rank from the local op structure
    (graph/dsl.py _static_rank), not from whole-graph shape inference."""
    import numpy as np
    from tensorframes_amd.graph import dsl
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, [None, 4], name="x")
        c = tf.constant(np.ones((3, 4)))
        m = tf.matmul(x, c, transpose_b=True)
        e = tf.expand_dims(tf.reduce_sum(tf.square(c), 1), 0)
        d = tf.tile(e, tf.stack([tf.shape(x)[0], 1])) + 2.0 * m
        a = tf.argmin(d, 1)
        r = tf.reduce_min(d, 1, keep_dims=True)
        s = tf.reshape(d, [-1])
        cands = [x, c, m, e, d, a, r, s, tf.cast(a, tf.float32), tf.reduce_sum(d, [0, 1])]
        ranks = [dsl._static_rank(t) for t in cands]
        calls = []
        orig = g._inferred
        g._inferred = lambda: calls.append(1) or orig()
        tot = tf.reduce_sum(tf.reduce_min(d, 1), name="tot")
        assert not calls
        g._inferred = orig
    assert ranks == [t.get_shape().ndims for t in cands] == [2, 2, 2, 2, 2, 1, 2, 1, 1, 0]
    assert tot.get_shape().ndims == 0

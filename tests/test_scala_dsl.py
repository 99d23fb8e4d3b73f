"""The Scala DSL vocabulary (tensorframes_amd.scala_dsl) on the reference's DSL
suites: constants, reduce, scoping, block/row placeholders, method-style
DataFrame ops (reference: src/test/scala/org/tensorframes/DSLOperationsSuite.scala:9-70,
src/test/scala/org/tensorframes/dsl/BasicSuite.scala:8-34)."""
import numpy as np

import tensorframes_amd as tfs
from tensorframes_amd import scala_dsl as dsl
from tensorframes_amd.graph import dsl as tf


def test_constant_add_map_blocks():
    df = tfs.create_dataframe([tfs.Row(x=float(i)) for i in range(5)])
    with dsl.with_graph():
        x = dsl.block(df, "x")
        z = dsl.add(x, dsl.constant(3.0), name="z")
        out = df.mapBlocks(z)
    np.testing.assert_allclose(out.to_numpy("z"), np.arange(5) + 3.0)


def test_reduce_blocks_sum_min():
    df = tfs.analyze(tfs.create_dataframe([tfs.Row(x=[float(i), -float(i)]) for i in range(6)]))
    with dsl.with_graph():
        xi = dsl.placeholder(tf.float64, dsl.Unknown, 2, name="x_input")
        s = df.reduceBlocks(dsl.reduce_sum(xi, [0], name="x"))
    np.testing.assert_allclose(s, [15.0, -15.0])
    with dsl.with_graph():
        xi = dsl.placeholder(tf.float64, dsl.Unknown, 2, name="x_input")
        m = df.reduceBlocks(dsl.reduce_min(xi, [0], name="x"))
    np.testing.assert_allclose(m, [0.0, -5.0])


def test_scope_names_and_fill():
    with dsl.with_graph() as g:
        with dsl.scope("outer"):
            c = dsl.zeros(3, name="z")
            f = dsl.fill([2, 2], 1.5, name="f")
            o = dsl.ones(2, dtype=tf.int32)
        assert c.name.startswith("outer/z") and f.name.startswith("outer/f")
        node = g.as_graph_def().node
        ops = {n.name: n.op for n in node}
        assert ops["outer/f"] == "Fill" and "outer/f/dims" in ops
        assert o.dtype == tf.int32


def test_row_placeholder_and_map_rows():
    df = tfs.analyze(tfs.create_dataframe([tfs.Row(y=[float(i), 1.0]) for i in range(4)]))
    with dsl.with_graph():
        y = dsl.row(df, "y")
        assert y.get_shape().as_list() == [2]
        out = df.mapRows(dsl.identity(dsl.reduce_sum(y, [0]), name="s"))
    np.testing.assert_allclose(out.to_numpy("s"), np.arange(4) + 1.0)

"""The reference's Scala graph DSL, in Python.

TensorFrames ships a small Scala DSL next to the Python API (reference:
src/main/scala/org/tensorframes/dsl/package.scala:16-132, DslImpl.scala,
Implicits.scala). A JVM does not exist here, so its vocabulary is offered on top of
the TF-1.x-compatible builder (`tensorframes_amd.tf`), which emits the same
GraphDef ops (Placeholder/Const/Fill/Identity/Add/Div/Sum/Min with `T`,
`Tidx=int32`, `keep_dims=false`):

    from tensorframes_amd import scala_dsl as dsl
    with dsl.with_graph():
        x = dsl.block(df, "x")
        out = df.mapBlocks(dsl.add(x, 3.0, name="z"))

Differences from the Scala DSL: ops are built eagerly into the current graph
(a `name=` argument replaces Scala's `.named(...)`), and `fill` takes dims of
any rank (the Scala version throws HighDimException above rank 1).
"""
from __future__ import annotations

import contextlib
from typing import Optional, Sequence

from . import core
from .frame.column_info import HighDimException  # noqa: F401  (re-exported, as in dsl/package.scala)
from .graph import dsl as tf

# unknown dimension (Shape.Unknown in the Scala DSL)
Unknown = -1


def _dims(shape: Sequence[int]):
    return [None if (d is None or d < 0) else int(d) for d in shape]


@contextlib.contextmanager
def with_graph():
    """Fresh graph with fresh name counters (Paths.withGraph, S/dsl/Paths.scala:40-55)."""
    g = tf.Graph()
    with g.as_default():
        yield g


withGraph = with_graph  # noqa: N816  (Scala spelling)


def scope(path_elem: str):
    """Name scope: nodes built inside are named `path_elem/...`."""
    return tf.name_scope(path_elem)


def placeholder(dtype, *shape: int, name: Optional[str] = None):
    return tf.placeholder(dtype, _dims(shape), name=name)


def constant(x, dtype=None, name: Optional[str] = None):
    """Scala literal types: a Double is float64, an Int int32 (the TF-Python
    default would make 3.0 a float32)."""
    if dtype is None:
        import numpy as np
        a = np.asarray(x)
        if a.dtype.kind == "f":
            dtype = tf.float64
        elif a.dtype.kind in "iu":
            dtype = tf.int32
    return tf.constant(x, dtype=dtype, name=name or "Const")


def fill(dims, value, name: Optional[str] = None):
    return tf.fill(dims, value, name=name)


def zeros(*shape: int, dtype=tf.float32, name: Optional[str] = None):
    return tf.zeros(list(shape), dtype=dtype, name=name)


def ones(*shape: int, dtype=tf.float32, name: Optional[str] = None):
    return tf.ones(list(shape), dtype=dtype, name=name)


def identity(op, name: Optional[str] = None):
    return tf.identity(op, name=name)


def add(x, y, name: Optional[str] = None):
    return tf.add(x, y, name=name)


def div(x, y, name: Optional[str] = None):
    return tf.div(x, y, name=name)


def reduce_sum(input_tensor, reduction_indices: Optional[Sequence[int]] = None, name: Optional[str] = None):
    return tf.reduce_sum(input_tensor, reduction_indices, name=name)


def reduce_min(input_tensor, reduction_indices: Optional[Sequence[int]] = None, name: Optional[str] = None):
    return tf.reduce_min(input_tensor, reduction_indices, name=name)


def block(df, col_name: str, tf_name: Optional[str] = None):
    return core.block(df, col_name, tf_name)


def row(df, col_name: str, tf_name: Optional[str] = None):
    return core.row(df, col_name, tf_name)

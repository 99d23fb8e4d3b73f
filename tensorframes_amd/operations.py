"""The operations interface, its default engine, shape hints and the
experimental operations.

* `ShapeDescription` — the shape-hint record passed with a graph: output
  shapes, requested fetches, placeholder -> column bindings
  (reference: src/main/scala/org/tensorframes/ShapeDescription.scala:12-20).
* `Operations` — the operation set every engine provides
  (reference: src/main/scala/org/tensorframes/Operations.scala:21-135,
  `OperationsInterface`), with `Ops`, the default engine that runs on the native
  executor (reference: src/main/scala/org/tensorframes/dsl/Ops.scala:12-51, which
  delegates to `DebugRowOps`). Each method takes a graph (DSL `Graph`,
  GraphDef bytes or a `.pb` path) plus a `ShapeDescription`, which is the Scala
  calling convention; the module-level functions in `core` are the Python one.
* `explain_detailed` / `convert_block_to_row` — the experimental operations
  (reference: src/main/scala/org/tensorframes/ExperimentalOperations.scala:12-23;
  `convertBlockToRow` is unimplemented (`???`) there and implemented here).
"""
from __future__ import annotations

import abc
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from . import core
from .frame.block import Block, is_dense
from .frame.column_info import ColumnInformation, DataFrameInfo
from .frame.dataframe import DataFrame, GroupedData, _Derived
from .frame.types import StructType
from .graph import dsl
from .utils.shape import UNKNOWN, Shape


@dataclass
class ShapeDescription:
    """out: tensor name -> shape hint; requested_fetches: the fetch names;
    inputs: placeholder path -> column name."""

    out: Dict[str, Shape] = field(default_factory=dict)
    requested_fetches: List[str] = field(default_factory=list)
    inputs: Dict[str, str] = field(default_factory=dict)

    @staticmethod
    def of(fetches, inputs: Optional[Dict[str, str]] = None) -> "ShapeDescription":
        """Hints of DSL tensors: the static shape of every fetch and of every
        zero-input node of their graph (reference: Node.hints,
        src/main/scala/org/tensorframes/dsl/Operation.scala:166-175; Python
        `_add_shapes`, src/main/python/tensorframes/core.py:52-72)."""
        fl = list(fetches) if isinstance(fetches, (list, tuple)) else [fetches]
        out: Dict[str, Shape] = {}
        names = []
        g = None
        for t in fl:
            if isinstance(t, dsl.Operation):
                t = t.outputs[0]
            g = t.graph
            names.append(t.name[:-2] if t.name.endswith(":0") else t.name)
            s = _shape_of(t)
            if s is not None:
                out[names[-1]] = s
        if g is not None:
            for op in g.get_operations():
                if not op.inputs and op.outputs and op.name not in out:
                    s = _shape_of(op.outputs[0])
                    if s is not None:
                        out[op.name] = s
        return ShapeDescription(out, names, dict(inputs or {}))


def _shape_of(t) -> Optional[Shape]:
    s = t.get_shape()
    if s.ndims is None:
        return None  # unknown rank: no hint
    return Shape([UNKNOWN if d is None else d for d in s.as_list()])


def _fetches(graph, hints: ShapeDescription):
    if not hints.requested_fetches:
        raise core.TensorFramesError("ShapeDescription.requested_fetches is empty: nothing to compute")
    return list(hints.requested_fetches)


class Operations(abc.ABC):
    """The TensorFrames operation set (reference: OperationsInterface,
    src/main/scala/org/tensorframes/Operations.scala:21-135)."""

    @abc.abstractmethod
    def map_rows(self, dataframe: DataFrame, graph, shape_hints: ShapeDescription) -> DataFrame: ...

    @abc.abstractmethod
    def map_blocks(self, dataframe: DataFrame, graph, shape_hints: ShapeDescription) -> DataFrame: ...

    @abc.abstractmethod
    def map_blocks_trimmed(self, dataframe: DataFrame, graph, shape_hints: ShapeDescription) -> DataFrame: ...

    @abc.abstractmethod
    def reduce_rows(self, dataframe: DataFrame, graph, shape_hints: ShapeDescription): ...

    @abc.abstractmethod
    def reduce_blocks(self, dataframe: DataFrame, graph, shape_hints: ShapeDescription): ...

    @abc.abstractmethod
    def aggregate(self, data: GroupedData, graph, shape_hints: ShapeDescription) -> DataFrame: ...

    @abc.abstractmethod
    def explain(self, df: DataFrame) -> str: ...


class Ops(Operations):
    """Default engine: the native GraphDef executor (GPU when available)."""

    def map_rows(self, dataframe, graph, shape_hints):
        return core.map_rows(_fetches(graph, shape_hints), dataframe, feed_dict=shape_hints.inputs or None,
                             graph=graph, shape_hints=shape_hints.out)

    def map_blocks(self, dataframe, graph, shape_hints):
        return core.map_blocks(_fetches(graph, shape_hints), dataframe, feed_dict=shape_hints.inputs or None,
                               graph=graph, shape_hints=shape_hints.out)

    def map_blocks_trimmed(self, dataframe, graph, shape_hints):
        return core.map_blocks(_fetches(graph, shape_hints), dataframe, trim=True,
                               feed_dict=shape_hints.inputs or None, graph=graph, shape_hints=shape_hints.out)

    def reduce_rows(self, dataframe, graph, shape_hints):
        return core.reduce_rows(_fetches(graph, shape_hints), dataframe, graph=graph, shape_hints=shape_hints.out)

    def reduce_blocks(self, dataframe, graph, shape_hints):
        return core.reduce_blocks(_fetches(graph, shape_hints), dataframe, graph=graph,
                                  shape_hints=shape_hints.out)

    def aggregate(self, data, graph, shape_hints):
        return core.aggregate(_fetches(graph, shape_hints), data, graph=graph, shape_hints=shape_hints.out)

    def explain(self, df):
        return core.explain(df)


ops = Ops()


# ------------------------------------------------------------------ experimental
def explain_detailed(df: DataFrame) -> DataFrameInfo:
    """Per-column tensor information (reference: ExperimentalOperations.scala:23)."""
    return DataFrameInfo.get(df.schema)


def convert_block_to_row(df: DataFrame) -> DataFrame:
    """Each partition (block) becomes ONE row whose cells are the whole block's
    column tensors: every column gains one leading dimension (reference:
    ExperimentalOperations.scala:13-21, declared there but left `???`). Empty
    partitions produce no row."""
    fields = []
    for f in df.schema.fields:
        stf = ColumnInformation(f).stf
        if stf is None:
            raise core.TensorFramesError(f"convert_block_to_row: column '{f.name}' is not a tensor column "
                                         f"({f.dataType})")
        # block shape [rows, *cell] -> cell of the new row; the new block is [1, rows, *cell]
        shape = Shape([UNKNOWN] + [UNKNOWN] + list(stf.shape.dims[1:]))
        fields.append(ColumnInformation.struct_field(f.name, stf.tf_dtype, shape))
    schema = StructType(fields)
    names = [f.name for f in df.schema.fields]

    def compute(blocks: Dict[int, Block]) -> Dict[int, Block]:
        res = {}
        for pid, b in blocks.items():
            if b.nrows == 0:
                res[pid] = Block(0, {n: torch.empty((0, 0)) for n in names})
                continue
            cols = {}
            for n in names:
                c = b.columns[n]
                if not is_dense(c):
                    raise core.TensorFramesError(f"convert_block_to_row: column '{n}' has cells of different "
                                                 f"shapes in partition {pid}")
                cols[n] = c.unsqueeze(0)
            res[pid] = Block(1, cols)
        return res

    return DataFrame(schema, _Derived(df, compute), df.num_partitions)


__all__ = ["ShapeDescription", "Operations", "Ops", "ops", "explain_detailed", "convert_block_to_row"]

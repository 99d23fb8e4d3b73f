"""Tensor information carried in column metadata.

Same metadata keys as the reference so schemas interoperate
(reference: src/main/scala/org/tensorframes/MetadataConstants.scala:19,27 — the
``org.spartf.shape`` typo is kept on purpose), same inference rule when the
metadata is absent (reference: src/main/scala/org/tensorframes/ColumnInformation.scala:124-138):
a numeric column is ``[?]``, ``array<numeric>`` is ``[?,?]`` and so on.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

from ..utils.shape import UNKNOWN, Shape
from .types import (ArrayType, DataType, NumericType, StructField, StructType, nested_array,
                    sql_type_for_tf, sql_type_from_string)

SHAPE_KEY = "org.spartf.shape"
TYPE_KEY = "org.sparktf.type"


class HighDimException(Exception):
    """Raised when a construct only supports tensors of low rank
    (reference: src/main/scala/org/tensorframes/Shape.scala:120-130)."""

    def __init__(self, shape):
        super().__init__(f"Shape {shape} is too high - tensorframes only supports dimensions <= 1 (vectors)")
        self.shape = shape


@dataclass(frozen=True)
class SparkTFColInfo:
    """Block shape (lead dim = rows) + scalar SQL type of a tensor column."""

    shape: Shape
    dataType: NumericType  # noqa: N815

    @property
    def tf_dtype(self) -> int:
        return self.dataType.tf_dtype

    def cell_shape(self) -> Shape:
        return self.shape.tail()


def _extract_from_type(dt: DataType) -> Optional[SparkTFColInfo]:
    if isinstance(dt, ArrayType):
        inner = _extract_from_type(dt.elementType)
        return None if inner is None else SparkTFColInfo(inner.shape.prepend(UNKNOWN), inner.dataType)
    if isinstance(dt, NumericType):
        return SparkTFColInfo(Shape(UNKNOWN), dt)
    return None


def _extract_from_metadata(meta: dict) -> Optional[SparkTFColInfo]:
    if SHAPE_KEY not in meta or TYPE_KEY not in meta:
        return None
    t = sql_type_from_string(meta[TYPE_KEY])
    if not isinstance(t, NumericType):
        return None
    return SparkTFColInfo(Shape(tuple(meta[SHAPE_KEY])), t)


class ColumnInformation:
    def __init__(self, field: StructField, stf: Optional[SparkTFColInfo] = None, _explicit=False):
        self.field = field
        if _explicit:
            self.stf = stf
        else:
            self.stf = _extract_from_metadata(field.metadata) or _extract_from_type(field.dataType)

    @staticmethod
    def with_info(field: StructField, info: Optional[SparkTFColInfo]) -> "ColumnInformation":
        return ColumnInformation(field, info, _explicit=True)

    @property
    def column_name(self) -> str:
        return self.field.name

    def merged(self) -> StructField:
        meta = dict(self.field.metadata)
        if self.stf is not None:
            meta[SHAPE_KEY] = list(self.stf.shape.dims)
            meta[TYPE_KEY] = str(self.stf.dataType)
        return self.field.copy(metadata=meta)

    @staticmethod
    def struct_field(name: str, tf_dtype: int, block_shape: Shape) -> StructField:
        """A non-nullable nested-array field with shape/type metadata
        (reference: ColumnInformation.scala:80-92)."""
        scalar = sql_type_for_tf(tf_dtype)
        f = StructField(name, nested_array(scalar, max(block_shape.num_dims - 1, 0)), nullable=False)
        return ColumnInformation.with_info(f, SparkTFColInfo(block_shape, scalar)).merged()

    def __eq__(self, o):
        return isinstance(o, ColumnInformation) and o.field == self.field and o.stf == self.stf

    def __repr__(self):
        return f"ColumnInformation({self.field!r}, {self.stf})"


class DataFrameInfo:
    """Tensor info of every column (reference: src/main/scala/org/tensorframes/DataFrameInfo.scala:7-39)."""

    def __init__(self, cols: List[ColumnInformation]):
        self.cols = cols

    @staticmethod
    def get(schema: StructType) -> "DataFrameInfo":
        return DataFrameInfo([ColumnInformation(f) for f in schema.fields])

    def explain(self) -> str:
        els = []
        for c in self.cols:
            if c.stf is not None:
                els.append(f"{c.stf.dataType}{c.stf.shape}")
            else:
                els.append(f"??{c.field.dataType}")
        return "DataFrame[" + ", ".join(els) + "]"

    def merged(self) -> StructType:
        return StructType([c.merged() for c in self.cols])

    __str__ = explain


def explain_schema(schema: StructType) -> str:
    """`print_schema` format (reference: src/main/scala/org/tensorframes/impl/DebugRowOps.scala:528-545)."""
    lines = ["root"]
    for c in DataFrameInfo.get(schema).cols:
        f = c.field
        line = f" |-- {f.name}: {f.dataType.typeName()} (nullable = {str(f.nullable).lower()})"
        if c.stf is not None:
            line += f" {c.stf.dataType.typeName()}{c.stf.shape}"
        else:
            line += " <no tensor info>"
        lines.append(line)
    return "\n".join(lines) + "\n"


def tf_scalar_of_field(field: StructField) -> Optional[int]:
    info = ColumnInformation(field).stf
    return None if info is None else info.tf_dtype


def sql_for_tf(enum: int) -> NumericType:
    return sql_type_for_tf(enum)

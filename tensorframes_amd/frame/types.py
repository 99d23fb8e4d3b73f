"""Spark-SQL-like schema types and `Row` for the tensorframes_amd DataFrame.

The reference runs on Spark DataFrames; there is no Spark here, so the frame
substrate carries its own small type system with the same names and the same
string forms (``typeName`` -> ``double``, ``toString`` -> ``DoubleType``), which
the tensor metadata uses (reference: src/main/scala/org/tensorframes/ColumnInformation.scala:16-26).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from ..utils import dtypes as D


class DataType:
    type_name = "data"

    def typeName(self) -> str:  # noqa: N802 (Spark naming)
        return self.type_name

    def simpleString(self) -> str:  # noqa: N802
        return self.type_name

    def __eq__(self, other):
        return type(self) is type(other)

    def __hash__(self):
        return hash(type(self).__name__)

    def __repr__(self):
        return type(self).__name__

    def __str__(self):
        return type(self).__name__


class NumericType(DataType):
    tf_dtype: int = D.DT_INVALID


class DoubleType(NumericType):
    type_name = "double"
    tf_dtype = D.DT_DOUBLE


class FloatType(NumericType):
    type_name = "float"
    tf_dtype = D.DT_FLOAT


class IntegerType(NumericType):
    type_name = "integer"
    tf_dtype = D.DT_INT32

    def simpleString(self):  # noqa: N802
        return "int"


class LongType(NumericType):
    type_name = "long"
    tf_dtype = D.DT_INT64

    def simpleString(self):  # noqa: N802
        return "bigint"


class UByteType(NumericType):
    """uint8 cells (decoded image pixels). An extension of the reference's
    four numeric types (its images entered as binary JPEG cells and were
    decoded to uint8 inside the graph: src/main/python/tensorframes_snippets/read_image.py:42);
    here a decoded uint8 column can be fed to a graph directly."""

    type_name = "ubyte"
    tf_dtype = D.DT_UINT8

    def simpleString(self):  # noqa: N802
        return "ubyte"


class BooleanType(DataType):
    type_name = "boolean"


class StringType(DataType):
    type_name = "string"


class BinaryType(DataType):
    type_name = "binary"


class ArrayType(DataType):
    type_name = "array"

    def __init__(self, elementType: DataType, containsNull: bool = False):  # noqa: N803
        self.elementType = elementType
        self.containsNull = containsNull

    def simpleString(self):  # noqa: N802
        return f"array<{self.elementType.simpleString()}>"

    def __eq__(self, other):
        return isinstance(other, ArrayType) and self.elementType == other.elementType

    def __hash__(self):
        return hash(("array", self.elementType))

    def __repr__(self):
        return f"ArrayType({self.elementType!r},{str(self.containsNull).lower()})"

    __str__ = __repr__


# the scalar types tensors can hold, in the reference's lookup order
# (reference: src/main/scala/org/tensorframes/impl/datatypes.scala:267)
SUPPORTED_SCALARS = [DoubleType(), FloatType(), IntegerType(), LongType(), UByteType()]

_BY_TF = {t.tf_dtype: t for t in SUPPORTED_SCALARS}
_BY_STR = {str(t): t for t in SUPPORTED_SCALARS}
_BY_STR.update({t.type_name: t for t in SUPPORTED_SCALARS})
_BY_STR["int"] = IntegerType()
_BY_STR["bigint"] = LongType()


def sql_type_for_tf(enum: int) -> NumericType:
    if enum not in _BY_TF:
        raise TypeError(f"TF dtype {D.dtype_name(enum)} has no supported SQL type "
                        f"(supported: double, float, int32, int64, uint8)")
    return _BY_TF[enum]


def sql_type_from_string(s: str) -> Optional[DataType]:
    return _BY_STR.get(s)


def scalar_type_of(dt: DataType) -> DataType:
    while isinstance(dt, ArrayType):
        dt = dt.elementType
    return dt


def array_depth(dt: DataType) -> int:
    n = 0
    while isinstance(dt, ArrayType):
        dt = dt.elementType
        n += 1
    return n


def nested_array(scalar: DataType, depth: int) -> DataType:
    t = scalar
    for _ in range(depth):
        t = ArrayType(t, containsNull=False)
    return t


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True,  # noqa: N803
                 metadata: Optional[Dict[str, Any]] = None):
        self.name = name
        self.dataType = dataType
        self.nullable = nullable
        self.metadata = dict(metadata or {})

    def copy(self, **kw) -> "StructField":
        d = dict(name=self.name, dataType=self.dataType, nullable=self.nullable,
                 metadata=dict(self.metadata))
        d.update(kw)
        return StructField(**d)

    def simpleString(self):  # noqa: N802
        return f"{self.name}:{self.dataType.simpleString()}"

    def __eq__(self, other):
        return (isinstance(other, StructField) and self.name == other.name and
                self.dataType == other.dataType and self.nullable == other.nullable and
                self.metadata == other.metadata)

    def __repr__(self):
        return f"StructField({self.name},{self.dataType!r},{str(self.nullable).lower()})"


class StructType(DataType):
    type_name = "struct"

    def __init__(self, fields: Optional[List[StructField]] = None):
        self.fields = list(fields or [])

    @property
    def names(self) -> List[str]:
        return [f.name for f in self.fields]

    fieldNames = names  # noqa: N815

    def __getitem__(self, key):
        if isinstance(key, int):
            return self.fields[key]
        for f in self.fields:
            if f.name == key:
                return f
        raise KeyError(f"No StructField named {key}")

    def __contains__(self, name):
        return any(f.name == name for f in self.fields)

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __eq__(self, other):
        return isinstance(other, StructType) and self.fields == other.fields

    def simpleString(self):  # noqa: N802
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def __repr__(self):
        return "StructType(List(" + ",".join(repr(f) for f in self.fields) + "))"


class Row(tuple):
    """A row with named fields; equality is positional (like pyspark's Row).

    ``Row(key='0', x=2.0)`` keeps the keyword order given.
    """

    __fields__: Optional[List[str]] = None  # per-schema subclasses set it once (see of_fields)

    def __new__(cls, *args, **kwargs):
        if args and kwargs:
            raise ValueError("Row takes positional or keyword values, not both")
        if kwargs:
            return tuple.__new__(Row.of_fields(tuple(kwargs)), list(kwargs.values()))
        return tuple.__new__(cls, args)

    @staticmethod
    def of_fields(names) -> type:
        """The Row class of one field list: a Row subclass whose field names
        live on the class, so its instances carry no per-row dict (the
        native row builder, runtime/packer.cpp build_rows, fills them in
        place)."""
        names = tuple(names)
        cls = _ROW_CLASSES.get(names)
        if cls is None:
            cls = type("Row", (Row,), {"__slots__": (), "__fields__": list(names), "__module__": Row.__module__})
            _ROW_CLASSES[names] = cls
        return cls

    @classmethod
    def from_fields(cls, names, values) -> "Row":
        return tuple.__new__(Row.of_fields(names), list(values))

    def asDict(self) -> Dict[str, Any]:  # noqa: N802
        if self.__fields__ is None:
            raise TypeError("Cannot convert a Row without field names to a dict")
        return dict(zip(self.__fields__, self))

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        fields = self.__fields__
        if fields is None or item not in fields:
            raise AttributeError(item)
        return tuple.__getitem__(self, fields.index(item))

    def __getitem__(self, item):
        if isinstance(item, str):
            fields = self.__fields__ or []
            if item not in fields:
                raise KeyError(item)
            return tuple.__getitem__(self, fields.index(item))
        return tuple.__getitem__(self, item)

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"

    def __reduce__(self):
        if self.__fields__ is None:
            return (Row, tuple(self))
        return (Row.from_fields, (self.__fields__, tuple(self)))


_ROW_CLASSES: Dict[tuple, type] = {}

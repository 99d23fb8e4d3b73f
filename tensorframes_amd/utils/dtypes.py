"""Scalar types: TF DataType enum <-> numpy <-> torch <-> SQL type names.

The supported tensor scalar types are the reference's
(reference: src/main/scala/org/tensorframes/impl/datatypes.scala:27-52,265-324):
double, float, int, long, plus binary for single-cell host inputs.
"""
from __future__ import annotations

import numpy as np
import torch

# TF DataType enum values (reference: src/main/protobuf/tensorflow/core/framework/types.proto)
DT_INVALID = 0
DT_FLOAT = 1
DT_DOUBLE = 2
DT_INT32 = 3
DT_UINT8 = 4
DT_INT16 = 5
DT_INT8 = 6
DT_STRING = 7
DT_INT64 = 9
DT_BOOL = 10
DT_BFLOAT16 = 14
DT_HALF = 19

_NP = {
    DT_FLOAT: np.float32,
    DT_DOUBLE: np.float64,
    DT_INT32: np.int32,
    DT_UINT8: np.uint8,
    DT_INT16: np.int16,
    DT_INT8: np.int8,
    DT_INT64: np.int64,
    DT_BOOL: np.bool_,
    DT_HALF: np.float16,
}
_TORCH = {
    DT_FLOAT: torch.float32,
    DT_DOUBLE: torch.float64,
    DT_INT32: torch.int32,
    DT_UINT8: torch.uint8,
    DT_INT16: torch.int16,
    DT_INT8: torch.int8,
    DT_INT64: torch.int64,
    DT_BOOL: torch.bool,
    DT_HALF: torch.float16,
    DT_BFLOAT16: torch.bfloat16,
}
_NAMES = {
    DT_FLOAT: "float32",
    DT_DOUBLE: "float64",
    DT_INT32: "int32",
    DT_UINT8: "uint8",
    DT_INT16: "int16",
    DT_INT8: "int8",
    DT_STRING: "string",
    DT_INT64: "int64",
    DT_BOOL: "bool",
    DT_BFLOAT16: "bfloat16",
    DT_HALF: "float16",
}


class DType:
    """A TF-style dtype object (what `tf.float32` & co. are in the DSL)."""

    __slots__ = ("enum",)

    def __init__(self, enum: int):
        self.enum = int(enum)

    @property
    def name(self) -> str:
        return _NAMES.get(self.enum, f"dtype({self.enum})")

    @property
    def as_numpy_dtype(self):
        return _NP[self.enum]

    @property
    def as_torch(self):
        return _TORCH[self.enum]

    @property
    def is_floating(self) -> bool:
        return self.enum in (DT_FLOAT, DT_DOUBLE, DT_HALF, DT_BFLOAT16)

    @property
    def is_integer(self) -> bool:
        return self.enum in (DT_INT32, DT_INT64, DT_INT16, DT_INT8, DT_UINT8)

    def __eq__(self, o):
        if isinstance(o, DType):
            return self.enum == o.enum
        try:
            return self.enum == as_dtype(o).enum
        except (TypeError, KeyError):
            return False

    def __hash__(self):
        return hash(self.enum)

    def __repr__(self):
        return f"tf.{self.name}"


float32 = DType(DT_FLOAT)
float64 = DType(DT_DOUBLE)
double = float64
int32 = DType(DT_INT32)
int64 = DType(DT_INT64)
uint8 = DType(DT_UINT8)
int16 = DType(DT_INT16)
int8 = DType(DT_INT8)
string = DType(DT_STRING)
bool_ = DType(DT_BOOL)
float16 = DType(DT_HALF)
bfloat16 = DType(DT_BFLOAT16)


def as_dtype(x) -> DType:
    if isinstance(x, DType):
        return x
    if isinstance(x, int) and not isinstance(x, bool):
        return DType(x)
    if isinstance(x, torch.dtype):
        for k, v in _TORCH.items():
            if v == x:
                return DType(k)
        raise TypeError(f"unsupported torch dtype {x}")
    if x is float:
        return float64
    if x is int:
        return int64
    if x is bool:
        return bool_
    if x is str or x is bytes:
        return string
    if isinstance(x, str):
        m = {"float": float32, "float32": float32, "double": float64, "float64": float64,
             "int32": int32, "int": int32, "int64": int64, "long": int64, "string": string,
             "bool": bool_, "uint8": uint8}
        if x in m:
            return m[x]
    try:
        nd = np.dtype(x)
    except TypeError:
        raise TypeError(f"cannot interpret {x!r} as a dtype")
    for k, v in _NP.items():
        if np.dtype(v) == nd:
            return DType(k)
    if nd.kind in ("U", "S", "O"):
        return string
    raise TypeError(f"unsupported dtype {x!r}")


def numpy_dtype(enum: int):
    return _NP[enum]


def torch_dtype(enum: int):
    return _TORCH[enum]


def dtype_name(enum: int) -> str:
    return _NAMES.get(enum, str(enum))

"""Tensor shapes with unknown dimensions.

Behaviour follows the reference's `Shape` (reference: src/main/scala/org/tensorframes/Shape.scala:16-109):
an unknown dim is -1, ``check_more_precise_than`` is the compatibility test
used when binding columns to placeholders, and the string form is ``[?,2]``.
"""
from __future__ import annotations

from typing import Iterable, Optional, Sequence

UNKNOWN = -1


class Shape:
    __slots__ = ("dims",)

    def __init__(self, *dims):
        if len(dims) == 1 and isinstance(dims[0], (list, tuple)):
            dims = tuple(dims[0])
        norm = []
        for d in dims:
            d = UNKNOWN if d is None else int(d)
            if d < UNKNOWN:
                raise ValueError(f"invalid dimension {d} in shape {dims}")
            norm.append(d)
        self.dims = tuple(norm)

    # -- constructors
    @staticmethod
    def empty() -> "Shape":
        return Shape(())

    @staticmethod
    def of(dims: Optional[Iterable]) -> Optional["Shape"]:
        return None if dims is None else Shape(tuple(dims))

    # -- properties
    @property
    def num_dims(self) -> int:
        return len(self.dims)

    ndims = num_dims

    def num_elements(self) -> Optional[int]:
        if any(d == UNKNOWN for d in self.dims):
            return None
        n = 1
        for d in self.dims:
            n *= d
        return n

    def has_unknown(self) -> bool:
        return any(d == UNKNOWN for d in self.dims)

    # -- transformations (reference: Shape.scala:37-49)
    def prepend(self, d) -> "Shape":
        return Shape((UNKNOWN if d is None else int(d),) + self.dims)

    def tail(self) -> "Shape":
        return Shape(self.dims[1:])

    def drop_inner(self) -> "Shape":
        return Shape(self.dims[:-1])

    def check_more_precise_than(self, other: "Shape") -> bool:
        """True if this shape is compatible with and at least as precise as `other`
        (same rank; every dim of `other` is unknown or equal)."""
        if other is None:
            return True
        if self.num_dims != other.num_dims:
            return False
        return all(o == UNKNOWN or s == o for s, o in zip(self.dims, other.dims))

    def merge(self, other: "Shape") -> Optional["Shape"]:
        """Least precise common shape (dims that disagree become unknown)."""
        if other.num_dims != self.num_dims:
            return None
        return Shape(tuple(a if a == b else UNKNOWN for a, b in zip(self.dims, other.dims)))

    def as_list(self):
        return [None if d == UNKNOWN else d for d in self.dims]

    def to_list(self):
        return list(self.dims)

    def __iter__(self):
        return iter(self.dims)

    def __len__(self):
        return len(self.dims)

    def __getitem__(self, i):
        return self.dims[i]

    def __eq__(self, other):
        if isinstance(other, Shape):
            return self.dims == other.dims
        if isinstance(other, (list, tuple)):
            return self.dims == Shape(other).dims
        return NotImplemented

    def __hash__(self):
        return hash(self.dims)

    def __str__(self):
        return "[" + ",".join("?" if d == UNKNOWN else str(d) for d in self.dims) + "]"

    def __repr__(self):
        return f"Shape{self}"


def shape_from_numpy(arr_shape: Sequence[int]) -> Shape:
    return Shape(tuple(int(d) for d in arr_shape))

"""Columnar partition storage.

A `Block` is one partition: a row count plus one column store per field.
Numeric columns whose cells share one shape are stored densely as a single
tensor ``[rows, *cell]`` (host memory, optionally page-locked for DMA, or
device memory when the frame is cached on the GPU). This replaces the
reference's boxed ``Row`` <-> ``java.nio`` buffer loops
(reference: src/main/scala/org/tensorframes/impl/DataOps.scala:20-81,
src/main/scala/org/tensorframes/impl/TFDataOps.scala:27-204): the tensor IS the block.
Ragged numeric columns keep one array per cell; other columns (strings,
binary, ...) are Python lists.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..utils import dtypes as D
from ..utils.shape import UNKNOWN, Shape


class RaggedColumn:
    """Numeric column whose cells have different shapes (one array per row)."""

    __slots__ = ("cells", "tf_dtype")

    def __init__(self, cells: List[np.ndarray], tf_dtype: int):
        self.cells = cells
        self.tf_dtype = tf_dtype

    def __len__(self):
        return len(self.cells)

    def take(self, idx) -> "RaggedColumn":
        return RaggedColumn([self.cells[i] for i in idx], self.tf_dtype)

    def slice(self, a, b) -> "RaggedColumn":
        return RaggedColumn(self.cells[a:b], self.tf_dtype)


class ObjectColumn:
    """Non-tensor column (strings, bytes, arbitrary Python values)."""

    __slots__ = ("values",)

    def __init__(self, values: List[Any]):
        self.values = list(values)

    def __len__(self):
        return len(self.values)

    def take(self, idx) -> "ObjectColumn":
        return ObjectColumn([self.values[i] for i in idx])

    def slice(self, a, b) -> "ObjectColumn":
        return ObjectColumn(self.values[a:b])


class StringColumn(ObjectColumn):
    """UTF-8 string (or binary) column in Arrow layout: int64 offsets [n+1]
    and one byte buffer, host or device tensors — no Python object per row.
    groupBy keys of this type are grouped on the device
    (ops/groupby.string_key_words); `values` decodes to Python str (or
    bytes) only when rows are materialised (collect)."""

    __slots__ = ("offsets", "data", "binary", "_values")

    def __init__(self, offsets: torch.Tensor, data: torch.Tensor, binary: bool = False):
        self.offsets = offsets
        self.data = data
        self.binary = binary
        self._values = None

    @staticmethod
    def from_values(values, binary: bool = False) -> "StringColumn":
        enc = [v if isinstance(v, (bytes, bytearray)) else str(v).encode("utf-8") for v in values]
        lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
        offs = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.frombuffer(b"".join(enc), dtype=np.uint8).copy()
        return StringColumn(torch.from_numpy(offs), torch.from_numpy(data), binary)

    @staticmethod
    def from_numpy(arr: np.ndarray) -> "StringColumn":
        """A numpy 'U' / 'S' array (fixed width) -> Arrow layout, vectorised."""
        binary = arr.dtype.kind == "S"
        b = arr if binary else np.char.encode(arr, "utf-8")
        b = np.ascontiguousarray(b)
        w = b.dtype.itemsize
        lens = np.char.str_len(b).astype(np.int64) if len(b) else np.zeros(0, np.int64)
        offs = np.zeros(len(b) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        if w == 0 or len(b) == 0:
            return StringColumn(torch.from_numpy(offs), torch.zeros(0, dtype=torch.uint8), binary)
        raw = b.view(np.uint8).reshape(len(b), w)
        mask = np.arange(w)[None, :] < lens[:, None]
        return StringColumn(torch.from_numpy(offs), torch.from_numpy(np.ascontiguousarray(raw[mask])), binary)

    def __len__(self):
        return int(self.offsets.shape[0]) - 1

    @property
    def values(self):
        if self._values is None:
            offs = self.offsets.cpu().numpy()
            raw = self.data.cpu().numpy().tobytes()
            base = int(offs[0]) if len(offs) else 0
            if self.binary:
                self._values = [raw[a - base:b - base] for a, b in zip(offs[:-1].tolist(), offs[1:].tolist())]
            else:
                self._values = [raw[a - base:b - base].decode("utf-8") for a, b in
                                zip(offs[:-1].tolist(), offs[1:].tolist())]
        return self._values

    @property
    def device(self):
        return self.data.device

    @property
    def is_cuda(self):
        return self.data.is_cuda

    def to(self, device) -> "StringColumn":
        device = torch.device(device)
        if self.data.device == device:
            return self
        return StringColumn(self.offsets.to(device), self.data.to(device), self.binary)

    def lengths(self) -> torch.Tensor:
        return self.offsets[1:] - self.offsets[:-1]

    def take(self, idx) -> "StringColumn":
        idx = np.asarray(idx, dtype=np.int64)
        offs = self.offsets.cpu().numpy()
        data = self.data.cpu().numpy()
        starts = offs[idx]
        lens = offs[idx + 1] - starts
        new = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(lens, out=new[1:])
        pos = np.repeat(starts - new[:-1], lens) + np.arange(new[-1], dtype=np.int64)
        return StringColumn(torch.from_numpy(new), torch.from_numpy(data[pos]), self.binary)

    def slice(self, a, b) -> "StringColumn":
        offs = self.offsets[a:b + 1]
        if offs.numel() == 0:
            return StringColumn(torch.zeros(1, dtype=torch.int64), self.data[:0], self.binary)
        lo, hi = int(offs[0]), int(offs[-1])
        return StringColumn(offs - lo, self.data[lo:hi], self.binary)


Column = Any  # torch.Tensor | RaggedColumn | ObjectColumn | StringColumn


@dataclass
class Block:
    nrows: int
    columns: Dict[str, Column] = field(default_factory=dict)

    def column(self, name: str) -> Column:
        return self.columns[name]

    def select(self, names: Sequence[str]) -> "Block":
        return Block(self.nrows, {n: self.columns[n] for n in names})

    def slice(self, a: int, b: int) -> "Block":
        return Block(b - a, {n: col_slice(c, a, b) for n, c in self.columns.items()})

    def take(self, idx) -> "Block":
        return Block(len(idx), {n: col_take(c, idx) for n, c in self.columns.items()})

    def to(self, device) -> "Block":
        return Block(self.nrows, {n: (c.to(device) if isinstance(c, (torch.Tensor, StringColumn)) else c)
                                  for n, c in self.columns.items()})


def is_dense(col: Column) -> bool:
    return isinstance(col, torch.Tensor)


def col_slice(col: Column, a: int, b: int) -> Column:
    if isinstance(col, torch.Tensor):
        return col[a:b]
    return col.slice(a, b)


def col_take(col: Column, idx) -> Column:
    if isinstance(col, torch.Tensor):
        t = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=col.device)
        return col.index_select(0, t)
    return col.take(list(idx))


def col_len(col: Column) -> int:
    return col.shape[0] if isinstance(col, torch.Tensor) else len(col)


def concat_columns(cols: List[Column]) -> Column:
    if all(isinstance(c, torch.Tensor) for c in cols):
        shapes = {tuple(c.shape[1:]) for c in cols}
        if len(shapes) == 1:
            return torch.cat([c.cpu() for c in cols], 0) if len(cols) > 1 else cols[0]
        cells = [np.asarray(x) for c in cols for x in c.cpu().numpy()]
        return RaggedColumn(cells, D.as_dtype(cols[0].dtype).enum)
    if all(isinstance(c, (torch.Tensor, RaggedColumn)) for c in cols):
        cells, dt = [], None
        for c in cols:
            if isinstance(c, torch.Tensor):
                dt = D.as_dtype(c.dtype).enum
                cells.extend(np.asarray(x) for x in c.cpu().numpy())
            else:
                dt = c.tf_dtype
                cells.extend(c.cells)
        return RaggedColumn(cells, dt)
    if cols and all(isinstance(c, StringColumn) for c in cols):
        if len(cols) == 1:
            return cols[0]
        offs, datas, base = [torch.zeros(1, dtype=torch.int64)], [], 0
        for c in cols:
            o = c.offsets.cpu()
            offs.append(o[1:] - o[0] + base)
            base += int(o[-1] - o[0])
            datas.append(c.data.cpu())
        return StringColumn(torch.cat(offs), torch.cat(datas) if datas else torch.zeros(0, dtype=torch.uint8),
                            cols[0].binary)
    vals = []
    for c in cols:
        vals.extend(column_values(c))
    return ObjectColumn(vals)


def concat_blocks(blocks: List[Block], names: Sequence[str]) -> Block:
    if not blocks:
        return Block(0, {})
    n = sum(b.nrows for b in blocks)
    return Block(n, {nm: concat_columns([b.columns[nm] for b in blocks]) for nm in names})


# ------------------------------------------------------------------ conversion

def _cell_shape(v) -> Optional[tuple]:
    """Shape of a nested-list / ndarray cell, None if ragged inside."""
    if isinstance(v, np.ndarray):
        return tuple(v.shape)
    if isinstance(v, (list, tuple)):
        if len(v) == 0:
            return (0,)
        subs = [_cell_shape(x) for x in v]
        if any(s is None for s in subs) or len(set(subs)) != 1:
            return None
        return (len(v),) + subs[0]
    return ()


def build_column(values: List[Any], tf_dtype: Optional[int]) -> Column:
    """Values of one column of one partition -> column store."""
    if tf_dtype is None or tf_dtype == D.DT_STRING:
        return ObjectColumn(values)
    npdt = D.numpy_dtype(tf_dtype)
    if len(values) == 0:
        return torch.empty((0,), dtype=D.torch_dtype(tf_dtype))
    shapes = {_cell_shape(v) for v in values}
    if None not in shapes and len(shapes) == 1:
        arr = np.asarray(values, dtype=npdt)
        return torch.from_numpy(np.asarray(arr, order="C"))
    return RaggedColumn([np.asarray(v, dtype=npdt) for v in values], tf_dtype)


def column_values(col: Column) -> List[Any]:
    """Column -> Python values (Spark-like: scalars, nested lists, str, bytes)."""
    if isinstance(col, torch.Tensor):
        t = col.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        return t.numpy().tolist()
    if isinstance(col, RaggedColumn):
        return [c.tolist() for c in col.cells]
    return list(col.values)


_NATIVE_ROW_KINDS = {"f": (4, 8), "i": (1, 2, 4, 8), "u": (1, 2, 4, 8), "b": (1,)}


def build_rows(names: Sequence[str], segments: Sequence[tuple]) -> list:
    """Row objects from column payloads, segment after segment: `segments` =
    [(nrows, [column payload per name])] with numpy arrays [rows, *cell],
    tensors or value lists. Built natively in one list (runtime/packer.cpp
    build_rows): scalars for rank-0 cells, nested lists for array cells
    (reference convertBack: DataOps.scala:20-61)."""
    import gc

    from .._native import _C
    from .types import Row
    cls = Row.of_fields(names)
    prepared = [(int(n), [_row_payload(c) for c in cols]) for n, cols in segments]
    # millions of new container objects: the cyclic GC would rescan them
    # every few hundred allocations (they cannot form cycles)
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _C.build_rows(cls, prepared)
    finally:
        if enabled:
            gc.enable()


def _row_payload(c: Any):
    if isinstance(c, torch.Tensor):
        c = c.detach().cpu()
        c = c.numpy() if c.dtype in _NUMPY_OK else column_values(c)
    if isinstance(c, np.ndarray):
        if c.dtype.kind in _NATIVE_ROW_KINDS and c.dtype.itemsize in _NATIVE_ROW_KINDS[c.dtype.kind] and c.ndim >= 1:
            return c
        return c.tolist() if c.dtype.kind != "O" else list(c)
    return c if isinstance(c, list) else list(c)


_NUMPY_OK = (torch.float32, torch.float64, torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8,
             torch.bool)


def column_cell(col: Column, i: int):
    if isinstance(col, torch.Tensor):
        v = col[i]
        return v.item() if v.dim() == 0 else v.cpu().numpy().tolist()
    if isinstance(col, RaggedColumn):
        return col.cells[i].tolist()
    return col.values[i]


def column_cell_shape(col: Column, i: int) -> Optional[Shape]:
    if isinstance(col, torch.Tensor):
        return Shape(tuple(col.shape[1:]))
    if isinstance(col, RaggedColumn):
        return Shape(tuple(col.cells[i].shape))
    return None


def column_tf_dtype(col: Column) -> Optional[int]:
    if isinstance(col, torch.Tensor):
        return D.as_dtype(col.dtype).enum
    if isinstance(col, RaggedColumn):
        return col.tf_dtype
    return None


def dense_block_shape(col: Column) -> Optional[Shape]:
    if isinstance(col, torch.Tensor):
        return Shape(tuple(col.shape))
    return None

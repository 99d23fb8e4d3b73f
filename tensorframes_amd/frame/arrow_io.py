"""Arrow and Parquet interop: the columnar data path into and out of frames.

The reference took its data from Spark DataFrames and packed rows into
tensors cell by cell (reference:
src/main/scala/org/tensorframes/impl/TFDataOps.scala:27-113,
src/main/scala/org/tensorframes/impl/datatypes.scala:60-152). Here columnar
Arrow buffers map straight onto block tensors:

* primitive numeric columns -> ``[rows]`` tensors (zero-copy, no nulls);
* ``fixed_size_list<...<numeric>>`` (nested to any depth) -> ``[rows, d1, d2, ...]``
  from the flat values buffer (zero-copy), shape recorded in the metadata;
* ``list<numeric>`` -> dense when every row has the same length, else a
  ragged column;
* ``string`` / ``binary`` -> object columns (e.g. JPEG bytes for map_rows).

Nulls are rejected, as everywhere in tensorframes_amd. Tensor metadata
(``org.spartf.shape`` / ``org.sparktf.type``) travels as Arrow field metadata,
so analysed shapes survive a Parquet round trip.

`read_parquet` is a lazy, distributed loader: Parquet row groups are dealt to
partitions, and each rank reads only the row groups of its own partitions
(p % world == rank), one partition at a time when the frame is streamed.
`DataFrame.write_parquet` writes one file per partition from the owning rank.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..parallel import dist
from ..utils import dtypes as D
from ..utils.shape import Shape
from .block import Block, ObjectColumn, RaggedColumn, StringColumn, column_values, is_dense
from .column_info import SHAPE_KEY, TYPE_KEY, ColumnInformation
from .types import BinaryType, StringType, StructField, StructType


def _pa():
    import pyarrow as pa
    return pa


_NUMERIC = {"float": D.DT_FLOAT, "double": D.DT_DOUBLE, "int32": D.DT_INT32, "int64": D.DT_INT64}


def _as_tensor(a: np.ndarray) -> torch.Tensor:
    """Zero-copy view of an Arrow-owned buffer (read-only: frames never
    write their inputs in place)."""
    import warnings
    a = np.ascontiguousarray(a)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return torch.from_numpy(a)


def _no_nulls(arr, name):
    if arr.null_count:
        raise ValueError(f"column '{name}' contains null values; tensorframes_amd requires non-null columns")


def _fixed_dims(t) -> Tuple[List[int], Any]:
    """(cell dims, value type) of a nest of fixed_size_list types."""
    pa = _pa()
    dims = []
    while pa.types.is_fixed_size_list(t):
        dims.append(t.list_size)
        t = t.value_type
    return dims, t


def _string_column(arr) -> StringColumn:
    """An Arrow string array as offsets + bytes (zero-copy views of its buffers
    where the layout allows)."""
    _, obuf, dbuf = arr.buffers()
    odt = np.int64 if _pa().types.is_large_string(arr.type) else np.int32
    offs = np.frombuffer(obuf, dtype=odt)[arr.offset:arr.offset + len(arr) + 1].astype(np.int64)
    data = np.frombuffer(dbuf, dtype=np.uint8) if dbuf is not None else np.zeros(0, np.uint8)
    lo, hi = (int(offs[0]), int(offs[-1])) if len(offs) else (0, 0)
    return StringColumn(torch.from_numpy(offs - lo), torch.from_numpy(data[lo:hi].copy()))


def _column_from_arrow(name: str, arr) -> Tuple[Any, StructField]:
    pa = _pa()
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    _no_nulls(arr, name)
    t = arr.type
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        # Arrow layout kept: offsets + bytes, no Python str per row
        return _string_column(arr), StructField(name, StringType(), False)
    if pa.types.is_binary(t) or pa.types.is_large_binary(t):
        return ObjectColumn([bytearray(v) for v in arr.to_pylist()]), StructField(name, BinaryType(), False)
    if str(t) in _NUMERIC:
        np_arr = arr.to_numpy(zero_copy_only=False)
        ten = _as_tensor(np_arr)
        return ten, ColumnInformation.struct_field(name, _NUMERIC[str(t)], Shape([-1]))
    if pa.types.is_fixed_size_list(t):
        dims, vt = _fixed_dims(t)
        if str(vt) not in _NUMERIC:
            raise TypeError(f"column '{name}': fixed_size_list of {vt} is not a tensor type")
        flat = arr
        for _ in dims:
            _no_nulls(flat, name)
            flat = flat.flatten()
        _no_nulls(flat, name)
        vals = flat.to_numpy(zero_copy_only=False)
        ten = _as_tensor(vals).reshape([len(arr)] + dims)
        return ten, ColumnInformation.struct_field(name, _NUMERIC[str(vt)], Shape([-1] + dims))
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        vt = t.value_type
        inner_dims, leaf = _fixed_dims(vt)
        if str(leaf) not in _NUMERIC:
            raise TypeError(f"column '{name}': list of {vt} is not a tensor type")
        offsets = arr.offsets.to_numpy()
        offsets = offsets - offsets[0]  # a sliced array's offsets index the parent buffer
        lengths = np.diff(offsets)
        flat = arr.flatten()
        for _ in inner_dims:
            flat = flat.flatten()
        _no_nulls(flat, name)
        vals = np.ascontiguousarray(flat.to_numpy(zero_copy_only=False))
        tf = _NUMERIC[str(leaf)]
        per = int(np.prod(inner_dims)) if inner_dims else 1
        if len(arr) and (lengths == lengths[0]).all():
            ten = _as_tensor(vals).reshape([len(arr), int(lengths[0])] + inner_dims)
            return ten, ColumnInformation.struct_field(name, tf, Shape([-1, -1] + inner_dims))
        cells = [vals[o * per:(o + ln) * per].reshape([ln] + inner_dims) for o, ln in zip(offsets[:-1], lengths)]
        return RaggedColumn(cells, tf), ColumnInformation.struct_field(name, tf, Shape([-1, -1] + inner_dims))
    raise TypeError(f"column '{name}': Arrow type {t} is not supported")


def _field_with_arrow_meta(f: StructField, meta: Optional[Dict[bytes, bytes]], nullable: bool) -> StructField:
    f = f.copy(nullable=nullable)
    if not meta:
        return f
    m = dict(f.metadata)
    for k in (SHAPE_KEY, TYPE_KEY):
        v = meta.get(k.encode())
        if v is not None:
            m[k] = json.loads(v.decode())
    return f.copy(metadata=m)


def block_from_arrow(table, names: Optional[Sequence[str]] = None) -> Tuple[Block, StructType]:
    cols, fields = {}, []
    for i, name in enumerate(names or table.column_names):
        col, f = _column_from_arrow(name, table.column(name))
        fld = table.schema.field(name)
        fields.append(_field_with_arrow_meta(f, fld.metadata, fld.nullable))
        cols[name] = col
    return Block(table.num_rows, cols), StructType(fields)


def from_arrow(table, num_partitions: Optional[int] = None):
    """DataFrame over an in-memory `pyarrow.Table` (or RecordBatch),
    partitions being zero-copy row slices."""
    from .dataframe import DataFrame, _bounds, _Materialized
    pa = _pa()
    if isinstance(table, pa.RecordBatch):
        table = pa.Table.from_batches([table])
    nparts = num_partitions or max(1, dist.world_size())
    n = table.num_rows
    blocks, schema = {}, None
    for p in dist.local_partitions(nparts):
        a, b = _bounds(n, nparts, p)
        blk, schema = block_from_arrow(table.slice(a, b - a))
        blocks[p] = blk
    if schema is None:
        schema = block_from_arrow(table.slice(0, 0))[1]
    return DataFrame(schema, _Materialized(blocks), nparts)


# ------------------------------------------------------------------ frame -> arrow
def _arrow_from_dense(t: torch.Tensor):
    pa = _pa()
    a = t.detach().cpu().contiguous().numpy()
    arr = pa.array(a.reshape(-1))
    for d in reversed(a.shape[1:]):
        arr = pa.FixedSizeListArray.from_arrays(arr, int(d))
    return arr


def _arrow_column(col, field: StructField):
    pa = _pa()
    if isinstance(col, torch.Tensor):
        return _arrow_from_dense(col)
    if isinstance(col, RaggedColumn):
        return pa.array([np.asarray(c).tolist() for c in col.cells])
    if isinstance(col, StringColumn) and not isinstance(field.dataType, BinaryType) and not col.binary:
        offs = col.offsets.cpu().numpy()
        data = pa.py_buffer(col.data.cpu().numpy())
        if len(offs) and int(offs[-1]) < (1 << 31):
            return pa.StringArray.from_buffers(len(col), pa.py_buffer(offs.astype(np.int32)), data)
        return pa.LargeStringArray.from_buffers(len(col), pa.py_buffer(offs.astype(np.int64)), data)
    vals = column_values(col)
    if isinstance(field.dataType, BinaryType):
        return pa.array([bytes(v) for v in vals], type=pa.binary())
    return pa.array(vals)


def _arrow_field(f: StructField, arr):
    pa = _pa()
    meta = {k.encode(): json.dumps(v).encode() for k, v in f.metadata.items() if k in (SHAPE_KEY, TYPE_KEY)}
    return pa.field(f.name, arr.type, nullable=f.nullable, metadata=meta or None)


def block_to_arrow(b: Block, schema: StructType):
    pa = _pa()
    arrays, fields = [], []
    for f in schema.fields:
        arr = _arrow_column(b.columns[f.name], f)
        arrays.append(arr)
        fields.append(_arrow_field(f, arr))
    return pa.Table.from_arrays(arrays, schema=pa.schema(fields))


def to_arrow(df):
    """All rows as one `pyarrow.Table` (gathered on every rank)."""
    pa = _pa()
    local = [(pid, block_to_arrow(b, df.schema)) for pid, b in df._iter_blocks()]
    parts = [x for chunk in dist.all_gather_object(local) for x in chunk]
    parts.sort(key=lambda x: x[0])
    tables = [t for _, t in parts]
    if not tables:
        return block_to_arrow(Block(0, {f.name: torch.empty(0) for f in df.schema.fields}), df.schema)
    return pa.concat_tables(tables)


# ------------------------------------------------------------------ parquet
def _parquet_files(path: str) -> List[str]:
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.parquet")))
        if not files:
            raise FileNotFoundError(f"no .parquet files under {path}")
        return files
    return [path]


def read_parquet(path: str, columns: Optional[Sequence[str]] = None, num_partitions: Optional[int] = None):
    """Lazy DataFrame over a Parquet file or a directory of them. Row groups
    are the unit of work: partition p reads its share of the row groups, on
    the rank that owns p only."""
    import pyarrow.parquet as pq
    from .dataframe import DataFrame, _Generated
    files = _parquet_files(path)
    units: List[Tuple[str, int]] = []
    for fpath in files:
        md = pq.ParquetFile(fpath).metadata
        units += [(fpath, g) for g in range(md.num_row_groups)]
    nparts = num_partitions or max(1, min(len(units), max(1, dist.world_size())) if units else 1)
    nparts = max(1, nparts)
    assign = [units[p * len(units) // nparts:(p + 1) * len(units) // nparts] for p in range(nparts)]
    # schema from the first file (row-group independent)
    first = pq.ParquetFile(files[0])
    arrow_schema = first.schema_arrow
    cols = list(columns) if columns else arrow_schema.names
    empty = arrow_schema.empty_table().select(cols)
    schema = block_from_arrow(empty)[1]

    def load(p: int) -> Block:
        import pyarrow as pa
        tables = []
        for fpath, g in assign[p]:
            tables.append(pq.ParquetFile(fpath).read_row_group(g, columns=cols))
        t = pa.concat_tables(tables) if tables else empty
        return block_from_arrow(t, cols)[0]
    return DataFrame(schema, _Generated(nparts, load), nparts)


def write_parquet(df, path: str, row_group_rows: int = 1 << 20) -> str:
    """One Parquet file per partition (``part-00003.parquet``), written by
    the rank owning the partition; ``_SUCCESS`` marks a complete write."""
    import pyarrow.parquet as pq
    os.makedirs(path, exist_ok=True)
    ok = os.path.join(path, "_SUCCESS")
    if dist.rank() == 0 and os.path.exists(ok):
        os.remove(ok)
    dist.barrier()
    for pid, b in df._iter_blocks():
        pq.write_table(block_to_arrow(b, df.schema), os.path.join(path, f"part-{pid:05d}.parquet"),
                       row_group_size=row_group_rows)
    dist.barrier()
    if dist.rank() == 0:
        with open(ok, "w") as f:
            f.write("ok\n")
    dist.barrier()
    return path


__all__ = ["from_arrow", "to_arrow", "read_parquet", "write_parquet", "block_from_arrow", "block_to_arrow"]

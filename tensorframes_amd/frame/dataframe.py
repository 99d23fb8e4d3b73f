"""A partitioned, lazily evaluated columnar DataFrame (the Spark substrate).

TensorFrames runs on Spark DataFrames (reference: README.md:3-9); Spark is not
available here, so this module provides the subset of DataFrame behaviour the
TensorFrames operators rely on (reference: SURVEY.md §2.4):

* a schema of `StructField`s whose metadata carries tensor shape/type info;
* an ordered list of partitions; operators are lazy and run when an action
  (`collect`, `count`, `first`, ...) forces them;
* `groupBy(...)` for keyed aggregation, `repartition`, `cache`/`persist`;
* SPMD distribution: under torch.distributed every rank holds the partitions
  ``p % world_size == rank``; actions gather results to every rank.

Dense numeric columns are stored as one tensor per partition (see block.py),
which can live in page-locked host memory (DMA source/target) or, after
`cache_on_device()`, in HBM.
"""
from __future__ import annotations

import math
import numbers
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch

from ..parallel import dist
from ..utils import dtypes as D
from .block import (Block, ObjectColumn, RaggedColumn, StringColumn, build_column, build_rows, column_values, concat_blocks,
                    is_dense)
from .column_info import ColumnInformation, DataFrameInfo, explain_schema
from .types import (ArrayType, BinaryType, BooleanType, DataType, DoubleType, FloatType, IntegerType,
                    LongType, NumericType, Row, StringType, StructField, StructType, scalar_type_of)


# ------------------------------------------------------------------ sources
class _Source:
    def compute(self) -> Dict[int, Block]:
        raise NotImplementedError


class _Materialized(_Source):
    def __init__(self, blocks: Dict[int, Block]):
        self._blocks = blocks

    def compute(self):
        return self._blocks


class _Failed(_Source):
    """A frame whose (eager) computation failed on this rank: the error is
    raised when an action evaluates it, inside the action's agreed local phase
    (parallel/dist.agreed), so every rank raises together."""

    def __init__(self, err: BaseException):
        self._err = err

    def compute(self):
        raise self._err


class _Generated(_Source):
    def __init__(self, num_partitions: int, fn: Callable[[int], Block]):
        self._n = num_partitions
        self._fn = fn

    def compute(self):
        return {p: self._fn(p) for p in dist.local_partitions(self._n)}


class _Derived(_Source):
    """Partitions computed from the parent's. `fn` maps any subset of the
    parent's local blocks {pid: block} to the same pids; when `streamable`,
    actions may evaluate partition by partition (bounded memory)."""

    def __init__(self, parent: "DataFrame", fn: Callable[[Dict[int, Block]], Dict[int, Block]],
                 streamable: bool = True):
        self._parent = parent
        self._fn = fn
        self.streamable = streamable

    def compute(self):
        return self._fn(self._parent._blocks())

    def iterate(self):
        """Streams the parent's partitions through fn in small groups: up to
        `Config.stream_group_bytes` of input per call, so a pipelined engine
        call spans several partitions (one H2D ramp-up per group, not per
        partition) while memory stays bounded."""
        from ..config import config
        from .. import engine
        group: Dict[int, Block] = {}
        nbytes = 0
        pending = None  # (group, results, completion handles) enqueued, not yet waited
        progs = set()
        try:
            for pid, b in self._parent._iter_blocks():
                group[pid] = b
                nbytes += _block_bytes(b)
                if nbytes >= config.stream_group_bytes or len(group) >= _MAX_GROUP_PARTITIONS:
                    # enqueue this group, THEN wait for (and hand out) the
                    # previous one: the chunk pipeline never drains between groups
                    nxt = self._start_group(group, progs)
                    if pending is not None:
                        yield from self._finish_group(pending)
                    pending = nxt
                    group, nbytes = {}, 0
            if group:
                nxt = self._start_group(group, progs)
                if pending is not None:
                    yield from self._finish_group(pending)
                pending = nxt
            if pending is not None:
                done, pending = pending, None
                yield from self._finish_group(done)
        finally:
            if pending is not None:
                engine.wait_pipelines(pending[2])
            for prog in progs:
                prog.release_pipeline()

    def _start_group(self, group: Dict[int, Block], progs: set):
        from .. import engine
        with engine.deferred_pipelines() as handles:
            res = self._fn(group)
        progs.update(h[0] for h in handles)
        return group, res, list(handles)

    def _finish_group(self, pending):
        from .. import engine
        group, res, handles = pending
        engine.wait_pipelines(handles)
        for pid in sorted(group):
            yield pid, res[pid]


_MAX_GROUP_PARTITIONS = 16  # bound for columns whose size is only estimated


def _block_bytes(b: Block) -> int:
    """Bytes of the block's tensor columns; other columns (strings, ragged
    cells) count 64 bytes per row."""
    n = 0
    for c in b.columns.values():
        n += c.numel() * c.element_size() if isinstance(c, torch.Tensor) else 64 * b.nrows
    return n


# ------------------------------------------------------------------ DataFrame
class DataFrame:
    def __init__(self, schema: StructType, source: _Source, num_partitions: int):
        self._schema = schema
        self._source = source
        self._nparts = num_partitions
        self._persist = False
        self._cached: Optional[Dict[int, Block]] = None

    # -- metadata
    @property
    def schema(self) -> StructType:
        return self._schema

    @property
    def columns(self) -> List[str]:
        return self._schema.names

    @property
    def dtypes(self):
        return [(f.name, f.dataType.simpleString()) for f in self._schema.fields]

    @property
    def num_partitions(self) -> int:
        return self._nparts

    def getNumPartitions(self) -> int:  # noqa: N802
        return self._nparts

    @property
    def rdd(self):
        return self  # `df.rdd.getNumPartitions()` compatibility

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{n}: {t}" for n, t in self.dtypes) + "]"

    def printSchema(self):  # noqa: N802
        print(explain_schema(self._schema), end="")

    def explain_tensors(self) -> str:
        """`DataFrame[double[?,2], ...]` (reference: src/main/scala/org/tensorframes/DataFrameInfo.scala:10-17)."""
        return DataFrameInfo.get(self._schema).explain()

    explainTensors = explain_tensors  # noqa: N815

    # -- evaluation
    def _blocks(self) -> Dict[int, Block]:
        if self._cached is not None:
            return self._cached
        b = self._source.compute()
        if self._persist:
            self._cached = b
        return b

    def _iter_blocks(self):
        """Local (pid, block) pairs in pid order, streamed through generated and
        streamable derived sources so only a bounded group of partitions
        (`Config.stream_group_bytes`) is alive at a time."""
        if self._cached is not None or self._persist:
            blocks = self._blocks()
            for pid in sorted(blocks):
                yield pid, blocks[pid]
            return
        src = self._source
        if isinstance(src, _Generated):
            for p in dist.local_partitions(src._n):
                yield p, src._fn(p)
        elif isinstance(src, _Derived) and src.streamable:
            yield from src.iterate()
        else:
            blocks = self._blocks()
            for pid in sorted(blocks):
                yield pid, blocks[pid]

    def foreach_block(self, fn: Callable[[int, Block], Any]) -> List[Any]:
        """Applies fn(pid, block) to every local partition, streaming (an action)."""
        return [fn(pid, b) for pid, b in self._iter_blocks()]

    def to_arrow(self):
        """All rows as a `pyarrow.Table` (frame/arrow_io.py)."""
        from .arrow_io import to_arrow
        return to_arrow(self)

    def write_parquet(self, path: str, row_group_rows: int = 1 << 20) -> str:
        """One Parquet file per partition under `path` (frame/arrow_io.py)."""
        from .arrow_io import write_parquet
        return write_parquet(self, path, row_group_rows)

    def write_checkpoint(self, path: str) -> str:
        """Write every partition + the schema under `path` (see frame/checkpoint.py)."""
        from .checkpoint import write_checkpoint
        return write_checkpoint(self, path)

    def cache(self) -> "DataFrame":
        self._persist = True
        return self

    def persist(self, *_args) -> "DataFrame":
        return self.cache()

    def unpersist(self) -> "DataFrame":
        self._persist = False
        self._cached = None
        return self

    def cache_on_device(self, device=None) -> "DataFrame":
        """Device-resident copy: dense columns moved to HBM once, reused by every
        following operator (iterative workloads do not re-cross PCIe)."""
        from ..engine import compute_device
        dev = torch.device(device) if device is not None else compute_device()
        blocks = {p: b.to(dev) for p, b in self._blocks().items()}
        df = DataFrame(self._schema, _Materialized(blocks), self._nparts)
        df._persist = True
        df._cached = blocks
        return df

    def to_host(self) -> "DataFrame":
        blocks = {p: b.to(torch.device("cpu")) for p, b in self._blocks().items()}
        return DataFrame(self._schema, _Materialized(blocks), self._nparts)

    def local_blocks(self) -> Dict[int, Block]:
        return self._blocks()

    # -- actions
    @staticmethod
    def _column_payload(col, a: int = 0, b: Optional[int] = None):
        """A column slice in a cheap-to-pickle form: dense columns as one numpy
        array (a buffer, not one object per cell), others as value lists."""
        if is_dense(col):
            t = col[a:b]
            return t.detach().cpu().numpy()
        return column_values(col)[a:b]

    def _rows_of(self, nrows: int, payload: Dict[str, Any]) -> List[Row]:
        """Row objects straight from the column buffers (native convertBack,
        runtime/packer.cpp build_rows; reference: DataOps.scala:20-61)."""
        return build_rows(self._schema.names, [(nrows, [payload[n] for n in self._schema.names])])

    def collect(self, to: Optional[int] = None) -> List[Row]:
        """All rows, in partition order, as Row objects built natively from the
        column buffers (runtime/packer.cpp build_rows).

        Across ranks the rows go to every rank (SPMD programs branch on the
        result, so every rank must see it) or, with `to=<rank>` (or
        `Config.collect_to`), only to that rank, the Spark driver's view
        (reference: ExperimentalOperations.scala:92); the others get [].
        Dense columns move as tensors (one padded gather per column), only
        ragged / string columns are pickled (parallel/frame_comm.py)."""
        from ..config import config
        from ..parallel import frame_comm
        names = self._schema.names
        if to is None and config.collect_to != "all":
            to = int(config.collect_to) if str(config.collect_to).isdigit() else 0
        # evaluated once, partition by partition; agreed across ranks (a rank
        # that fails makes every rank raise, none waits in the gather)
        local = dist.agreed("collect", lambda: list(self._iter_blocks()))
        if not dist.is_distributed():
            return build_rows(names, [(b.nrows, [self._column_payload(b.columns[n]) for n in names])
                                      for _, b in local if b.nrows])
        parts = frame_comm.gather_blocks(local, names, self._schema, self._nparts, root=to)
        if parts is None:
            return []
        return build_rows(names, [(nrows, cols) for _, nrows, cols in parts])

    def count(self) -> int:
        """Rows over all ranks: one int64 all-reduce."""
        n = torch.tensor([dist.agreed("count", lambda: sum(b.nrows for _, b in self._iter_blocks()))],
                         dtype=torch.int64)
        return int(dist.all_reduce_host_(n, "Sum").item())

    def first(self) -> Optional[Row]:
        rows = self.take(1)
        return rows[0] if rows else None

    head = first

    def take(self, n: int) -> List[Row]:
        """The first n rows in partition order. Partitions are evaluated in
        order and evaluation stops once n rows are in hand (later partitions
        are never computed); across ranks, each partition's owner broadcasts
        only the rows still needed, dense columns as tensors."""
        if n <= 0:
            return []
        from ..parallel import frame_comm
        got = frame_comm.take_rows(self._iter_blocks(), self._schema.names, self._schema, self._nparts, n)
        return build_rows(self._schema.names, got)[:n]

    def show(self, n: int = 20):
        rows = self.take(n)
        print(" | ".join(self.columns))
        for r in rows:
            print(" | ".join(str(v) for v in r))

    def toPandas(self):  # noqa: N802
        import pandas as pd
        rows = self.collect()
        return pd.DataFrame([list(r) for r in rows], columns=self.columns)

    def to_numpy(self, column: str) -> np.ndarray:
        """All rows of a column as one array, on every rank (dense columns are
        gathered as tensors)."""
        from ..parallel import frame_comm
        blocks = dist.agreed("to_numpy", self._blocks)
        local = [(pid, blocks[pid]) for pid in sorted(blocks)]
        if not dist.is_distributed():
            parts = [(pid, b.nrows, [self._column_payload(b.columns[column])]) for pid, b in local if b.nrows]
        else:
            parts = frame_comm.gather_blocks(local, [column], self._schema, self._nparts)
        arrs = [c[0] if isinstance(c[0], np.ndarray) else np.asarray(c[0], dtype=object) for _, _, c in parts]
        return np.concatenate(arrs, 0) if arrs else np.zeros((0,))

    # -- transformations
    def select(self, *cols) -> "DataFrame":
        names = [c for cs in cols for c in (cs if isinstance(cs, (list, tuple)) else [cs])]
        for n in names:
            if n not in self._schema:
                raise ValueError(f"Column {n} not found in {self.columns}")
        schema = StructType([self._schema[n] for n in names])
        return DataFrame(schema, _Derived(self, lambda bs: {p: b.select(names) for p, b in bs.items()}),
                         self._nparts)

    def drop(self, *names) -> "DataFrame":
        return self.select([n for n in self.columns if n not in names])

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":  # noqa: N802
        fields = [f.copy(name=new) if f.name == existing else f for f in self._schema.fields]

        def fn(bs):
            return {p: Block(b.nrows, {(new if k == existing else k): v for k, v in b.columns.items()})
                    for p, b in bs.items()}
        return DataFrame(StructType(fields), _Derived(self, fn), self._nparts)

    def with_schema(self, schema: StructType) -> "DataFrame":
        """Same data, new schema (used by `analyze` to attach metadata)."""
        df = DataFrame(schema, _Derived(self, lambda bs: bs), self._nparts)
        return df

    def repartition(self, n: int) -> "DataFrame":
        """n even partitions in row order. Each rank receives only the rows of
        the partitions it owns: dense columns in one all-to-all per column
        (RCCL for device-resident frames), other columns pickled."""
        from ..parallel import frame_comm
        names = self.columns
        nin = self._nparts

        def fn(bs):
            return frame_comm.repartition_blocks(bs, names, self._schema, nin, n)
        return DataFrame(self._schema, _Derived(self, fn, streamable=False), n)

    def coalesce(self, n: int) -> "DataFrame":
        return self.repartition(min(n, self._nparts))

    def groupBy(self, *cols) -> "GroupedData":  # noqa: N802
        names = [c for cs in cols for c in (cs if isinstance(cs, (list, tuple)) else [cs])]
        for n in names:
            if n not in self._schema:
                raise ValueError(f"groupBy: column {n} not found in {self.columns}")
        return GroupedData(self, names)

    groupby = groupBy

    # -- TensorFrames method forms (reference: src/main/scala/org/tensorframes/dsl/Implicits.scala:25-116)
    def map_blocks(self, fetches, trim: bool = False, **kw) -> "DataFrame":
        from .. import core
        return core.map_blocks(fetches, self, trim=trim, **kw)

    mapBlocks = map_blocks  # noqa: N815

    def map_blocks_trimmed(self, fetches, **kw) -> "DataFrame":
        from .. import core
        return core.map_blocks(fetches, self, trim=True, **kw)

    mapBlocksTrimmed = map_blocks_trimmed  # noqa: N815

    def map_rows(self, fetches, feed_dict=None, **kw) -> "DataFrame":
        from .. import core
        return core.map_rows(fetches, self, feed_dict=feed_dict, **kw)

    mapRows = map_rows  # noqa: N815

    def reduce_blocks(self, fetches, **kw):
        from .. import core
        return core.reduce_blocks(fetches, self, **kw)

    reduceBlocks = reduce_blocks  # noqa: N815

    def reduce_rows(self, fetches, **kw):
        from .. import core
        return core.reduce_rows(fetches, self, **kw)

    reduceRows = reduce_rows  # noqa: N815

    def analyze(self) -> "DataFrame":
        from .. import core
        return core.analyze(self)

    def block(self, col_name: str, tf_name: Optional[str] = None):
        from .. import core
        return core.block(self, col_name, tf_name)

    def row(self, col_name: str, tf_name: Optional[str] = None):
        from .. import core
        return core.row(self, col_name, tf_name)


class GroupedData:
    def __init__(self, df: DataFrame, keys: List[str]):
        self.df = df
        self.keys = keys

    def aggregate(self, fetches, **kw) -> DataFrame:
        from .. import core
        return core.aggregate(fetches, self, **kw)

    def count(self) -> DataFrame:
        """Rows per key: the keys plus a column of ones go through `aggregate`
        with a Sum graph (device factorisation + segmented sum, keyed
        all-to-all across ranks); no rows are collected."""
        from .. import core, engine
        from ..graph import dsl as tf
        keys = list(self.keys)

        def fn(bs):
            out = {}
            for p, b in bs.items():
                kc = b.columns[keys[0]]
                dev = kc.device if isinstance(kc, torch.Tensor) else torch.device("cpu")
                cols = {k: b.columns[k] for k in keys}
                cols["count"] = engine.device_full(b.nrows, 1, torch.int64, dev)
                out[p] = Block(b.nrows, cols)
            return out
        fields = [self.df.schema[k] for k in keys] + [tensor_field("count", D.DT_INT64, [])]
        ones = DataFrame(StructType(fields), _Derived(self.df, fn), self.df._nparts)
        with tf.Graph().as_default():
            ci = tf.placeholder(tf.int64, [None], name="count_input")
            return core.aggregate(tf.reduce_sum(ci, [0], name="count"), ones.groupBy(*keys))


def _sort_key(k):
    return tuple((0, v) if isinstance(v, numbers.Number) else (1, str(v)) for v in k)


# ------------------------------------------------------------------ construction
def _bounds(n: int, parts: int, p: int):
    """Row range of partition p when n rows are sliced evenly (Spark parallelize)."""
    return (p * n) // parts, ((p + 1) * n) // parts


def _infer_type(v) -> Optional[DataType]:
    if v is None:
        return None
    if isinstance(v, (bool, np.bool_)):
        return BooleanType()
    if isinstance(v, np.generic):
        return {np.dtype(np.float64): DoubleType(), np.dtype(np.float32): FloatType(),
                np.dtype(np.int32): IntegerType(), np.dtype(np.int64): LongType()}.get(v.dtype, DoubleType())
    if isinstance(v, float):
        return DoubleType()
    if isinstance(v, int):
        return LongType()
    if isinstance(v, str):
        return StringType()
    if isinstance(v, (bytes, bytearray)):
        return BinaryType()
    if isinstance(v, np.ndarray):
        t = _infer_type(v.reshape(-1)[0]) if v.size else DoubleType()
        for _ in range(v.ndim):
            t = ArrayType(t, False)
        return t
    if isinstance(v, (list, tuple)):
        inner = None
        for x in v:
            inner = _infer_type(x)
            if inner is not None:
                break
        return ArrayType(inner or DoubleType(), False)
    raise TypeError(f"cannot infer a column type for value {v!r} of type {type(v).__name__}")


def _tf_of(dt: DataType) -> Optional[int]:
    s = scalar_type_of(dt)
    return s.tf_dtype if isinstance(s, NumericType) else None


def _normalize_rows(data: Sequence[Any], names: Optional[List[str]]):
    rows = data if isinstance(data, list) else list(data)
    if not rows:
        return [], names or []
    r0 = rows[0]
    if isinstance(r0, Row) and r0.__fields__:
        names = names or list(r0.__fields__)
        return rows, names  # Rows are tuples already: no per-row copy
    if isinstance(r0, dict):
        names = names or list(r0.keys())
        return [tuple(r[n] for n in names) for r in rows], names
    if isinstance(r0, tuple):
        names = names or [f"_{i + 1}" for i in range(len(r0))]
        return rows, names
    if isinstance(r0, list):
        names = names or [f"_{i + 1}" for i in range(len(r0))]
        return [tuple(r) for r in rows], names
    names = names or ["value"]
    return [(r,) for r in rows], names


def _validate_all_rows(rows: List[tuple], st: StructType) -> None:
    """Width and null checks over ALL rows. In a multi-rank job every rank
    holds the same local `rows` but packs only its own partitions; checking
    the whole list first makes a bad row fail on every rank before any rank
    enters a collective (instead of one rank raising while the rest block)."""
    ncols = len(st.fields)
    bad = next((r for r in rows if len(r) != ncols), None)
    if bad is not None:
        raise ValueError(f"row {bad} has {len(bad)} values, schema has {ncols} columns")
    for i, f in enumerate(st.fields):
        if any(r[i] is None for r in rows):
            raise ValueError(f"column '{f.name}' contains null values; tensorframes_amd requires "
                             f"non-null columns (the reference silently accepted them)")


def create_dataframe(data, schema=None, num_partitions: Optional[int] = None) -> DataFrame:
    """Build a DataFrame from local data (rows, dicts, tuples, scalars, or a
    dict of column arrays). `schema`: a StructType, a list of column names, or None."""
    nparts = num_partitions or max(1, dist.world_size())
    if isinstance(data, dict):
        return from_columns(data, num_partitions=nparts, schema=schema if isinstance(schema, StructType) else None)
    import sys
    pd = sys.modules.get("pandas")  # a pandas frame can only exist if pandas is loaded
    if pd is not None:
        if isinstance(data, pd.DataFrame):
            return from_columns({c: data[c].to_numpy() if data[c].dtype != object else list(data[c])
                                 for c in data.columns}, num_partitions=nparts)
    names = schema if isinstance(schema, (list, tuple)) else None
    rows, names = _normalize_rows(data, list(names) if names else None)
    if isinstance(schema, StructType):
        st = schema
        names = st.names
    else:
        fields = []
        for i, n in enumerate(names):
            t = None
            for r in rows:
                t = _infer_type(r[i])
                if t is not None:
                    break
            if t is None:
                t = StringType()
            fields.append(StructField(n, t, True))
        st = StructType(fields)
    if not isinstance(rows, list):
        rows = list(rows)
    ncols = len(names)
    blocks = {}
    n = len(rows)
    if dist.world_size() > 1:
        _validate_all_rows(rows, st)  # every rank raises, not only the owner of the bad row
    from .._native import _C
    for p in dist.local_partitions(nparts):
        a, b = _bounds(n, nparts, p)
        cols = {}
        for i, f in enumerate(st.fields):
            tf = _tf_of(f.dataType)
            packed = None
            if tf is not None:
                # native pass over the row tuples (also checks widths and nulls)
                try:
                    packed = _C.pack_column(rows, i, ncols, a, b, tf)
                except ValueError as e:
                    if "wrong width" in str(e):
                        bad = next(r for r in rows[a:b] if len(r) != ncols)
                        raise ValueError(f"row {bad} has {len(bad)} values, schema has {ncols} columns")
                    raise ValueError(f"column '{f.name}' contains null values; tensorframes_amd requires "
                                     f"non-null columns (the reference silently accepted them)")
            if packed is not None:
                cols[f.name] = packed
                continue
            for r in rows[a:b]:
                if len(r) != ncols:
                    raise ValueError(f"row {r} has {len(r)} values, schema has {ncols} columns")
            vals = [r[i] for r in rows[a:b]]
            if any(v is None for v in vals):
                raise ValueError(f"column '{f.name}' contains null values; tensorframes_amd requires "
                                 f"non-null columns (the reference silently accepted them)")
            cols[f.name] = build_column(vals, tf)
        blocks[p] = Block(b - a, cols)
    return DataFrame(st, _Materialized(blocks), nparts)


createDataFrame = create_dataframe  # noqa: N816


def _field_for_array(name: str, arr) -> StructField:
    """Dense whole-column arrays know their cell shape: record it in the
    metadata (lead dim unknown), so no `analyze` pass is needed."""
    if isinstance(arr, StringColumn):
        return StructField(name, BinaryType() if arr.binary else StringType(), False)
    if isinstance(arr, torch.Tensor):
        tf = D.as_dtype(arr.dtype).enum
        shape = tuple(arr.shape)
    else:
        arr = np.asarray(arr)
        if arr.dtype.kind in ("U", "S", "O"):
            return StructField(name, StringType() if arr.dtype.kind != "S" else BinaryType(), False)
        tf = D.as_dtype(arr.dtype).enum
        shape = tuple(arr.shape)
    return tensor_field(name, tf, shape[1:])


def tensor_field(name: str, dtype, cell_shape: Sequence[Optional[int]] = ()) -> StructField:
    """A tensor column field: nested arrays of a numeric type with the block
    shape ``[?, *cell_shape]`` in the metadata."""
    from ..utils.shape import Shape
    tf = D.as_dtype(dtype).enum
    dims = [-1] + [-1 if d is None else int(d) for d in cell_shape]
    return ColumnInformation.struct_field(name, tf, Shape(dims))


def from_columns(columns: Dict[str, Any], num_partitions: Optional[int] = None,
                 schema: Optional[StructType] = None, pinned: bool = False) -> DataFrame:
    """DataFrame from whole-column arrays ``{name: array[rows, *cell]}`` (zero-copy
    for contiguous numpy/torch inputs; `pinned=True` page-locks dense columns)."""
    nparts = num_partitions or max(1, dist.world_size())
    cols = {}
    n = None
    for k, v in columns.items():
        if isinstance(v, (torch.Tensor, StringColumn)):
            t = v
        else:
            a = np.asarray(v)
            if a.dtype.kind in ("U", "S") and a.ndim == 1:
                t = a  # fixed-width strings: Arrow-layout StringColumn per partition, vectorised
            else:
                t = torch.from_numpy(np.asarray(a, order="C")) if a.dtype.kind not in ("U", "S", "O") else list(v)
        ln = t.shape[0] if isinstance(t, (torch.Tensor, np.ndarray)) else len(t)  # StringColumn: rows
        if n is None:
            n = ln
        elif ln != n:
            raise ValueError(f"column {k} has {ln} rows, expected {n}")
        cols[k] = t
    n = n or 0
    st = schema or StructType([_field_for_array(k, v) for k, v in cols.items()])
    blocks = {}
    for p in dist.local_partitions(nparts):
        a, b = _bounds(n, nparts, p)
        bc = {}
        for k, t in cols.items():
            if isinstance(t, torch.Tensor):
                s = t[a:b]
                if pinned:
                    from ..engine import pin
                    s = pin(s)
                bc[k] = s
            elif isinstance(t, np.ndarray):
                bc[k] = StringColumn.from_numpy(t[a:b])
            elif isinstance(t, StringColumn):
                bc[k] = t.slice(a, b)
            else:
                bc[k] = ObjectColumn(t[a:b])
        blocks[p] = Block(b - a, bc)
    return DataFrame(st, _Materialized(blocks), nparts)


def generate(schema: StructType, num_partitions: int, fn: Callable[[int], Block]) -> DataFrame:
    """Lazily generated partitions (synthetic data sets larger than host RAM are
    produced partition by partition, only on the owning rank)."""
    return DataFrame(schema, _Generated(num_partitions, fn), num_partitions)


def range_(n: int, num_partitions: Optional[int] = None, name: str = "id") -> DataFrame:
    """DataFrame of one int64 column `id` = 0..n-1, generated lazily per
    partition (Spark's `sqlContext.range`, used by the reference's perf suite)."""
    nparts = num_partitions or max(1, dist.world_size())

    def fn(p):
        a, b = _bounds(n, nparts, p)
        return Block(b - a, {name: torch.arange(a, b, dtype=torch.int64)})
    return generate(StructType([StructField(name, LongType(), False)]), nparts, fn)

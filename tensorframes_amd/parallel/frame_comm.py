"""Frame-level data movement between ranks, scaled by rows, not by ranks.

The reference moves rows with Spark: `collect` brings them to the driver
(reference: src/main/scala/org/tensorframes/ExperimentalOperations.scala:92,
src/main/scala/org/tensorframes/impl/PythonInterface.scala:165-169) and
`repartition` is a shuffle. Here every rank runs the same program (SPMD) and
owns partitions p % world:

* dense columns (one dtype and cell shape on every rank) travel as tensors:
  a padded all_gather / gather for `collect`, one all_to_all per column for
  `repartition`, a broadcast for `take`; only ragged / string columns are
  pickled;
* whether a column is dense is read from the schema (analyzed block shape)
  and confirmed with one small integer all-reduce; the per-column metadata is
  exchanged only for columns the schema does not pin;
* partition sizes are agreed with one int64 all-reduce.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import dist

Kind = Optional[Tuple[torch.dtype, tuple]]  # (dtype, cell shape) of a dense column; None: object column


def _schema_kind(field) -> Kind:
    from ..frame.column_info import ColumnInformation
    from ..utils import dtypes as D
    stf = ColumnInformation(field).stf
    if stf is None or stf.shape.num_dims < 1:
        return None
    cell = stf.shape.tail()
    if cell.has_unknown():
        return None
    try:
        return D.torch_dtype(stf.tf_dtype), tuple(int(d) for d in cell.dims)
    except (KeyError, TypeError, ValueError):
        return None


def _schema_tf(field) -> Optional[int]:
    from ..frame.column_info import ColumnInformation
    stf = ColumnInformation(field).stf
    return stf.tf_dtype if stf is not None else None


def _local_kind(blocks: Sequence, name: str):
    """'none' (no local rows), (dtype, cell) when every local block holds a
    dense tensor of one dtype/cell, else 'obj'."""
    from ..frame.block import is_dense
    kinds = set()
    for b in blocks:
        if not b.nrows:
            continue
        c = b.columns[name]
        if not is_dense(c):
            return "obj"
        kinds.add((c.dtype, tuple(c.shape[1:])))
    if not kinds:
        return "none"
    return kinds.pop() if len(kinds) == 1 else "obj"


def column_kinds(blocks: Sequence, names: Sequence[str], schema) -> Dict[str, Kind]:
    """Per column: (dtype, cell shape) if it is dense on EVERY rank, else None.
    Collective (every rank calls it with its local blocks)."""
    local = {n: _local_kind(blocks, n) for n in names}
    if not dist.is_distributed():
        return {n: (k if isinstance(k, tuple) else None) for n, k in local.items()}
    out: Dict[str, Kind] = {}
    pinned = {n: _schema_kind(schema[n]) for n in names}
    cand = [n for n in names if pinned[n] is not None]
    if cand:
        ok = torch.tensor([int(local[n] == "none" or local[n] == pinned[n]) for n in cand], dtype=torch.int64)
        dist.all_reduce_host_(ok, "Min")
        for n, f in zip(cand, ok.tolist()):
            if f:
                out[n] = pinned[n]
    for n in names:  # string fields: never dense (their own tensor path), nothing to exchange
        if n not in out and _is_string_field(schema[n]):
            out[n] = None
    rest = [n for n in names if n not in out]
    if rest:
        # the schema does not pin these: a small metadata exchange (no data)
        metas = dist.all_gather_object([(str(local[n][0]), local[n][1]) if isinstance(local[n], tuple)
                                        else local[n] for n in rest])
        for j, n in enumerate(rest):
            ms = [m[j] for m in metas if m[j] != "none"]
            if ms and all(isinstance(m, tuple) for m in ms) and len(set(ms)) == 1:
                out[n] = (getattr(torch, ms[0][0].split(".")[-1]), tuple(ms[0][1]))
            elif not ms and isinstance(local[n], tuple):
                out[n] = local[n]
            else:
                out[n] = None
    return out


def _empty_strings(binary: bool):
    from ..frame.block import StringColumn
    return StringColumn.from_values([], binary)


def partition_rows(local: Dict[int, int], nparts: int) -> List[int]:
    """Rows of every partition (agreed by one int64 all-reduce)."""
    counts = torch.zeros(max(nparts, 1), dtype=torch.int64)
    for p, n in local.items():
        counts[p] = int(n)
    dist.all_reduce_host_(counts, "Sum")
    return counts.tolist()[:nparts]


def _host_cat(cols: List[Any], kind: Kind) -> torch.Tensor:
    ts = [c.detach().cpu() for c in cols]
    if not ts:
        return torch.empty((0,) + kind[1], dtype=kind[0])
    return ts[0].contiguous() if len(ts) == 1 else torch.cat(ts, 0)


def _is_string_field(field) -> bool:
    from ..frame.types import StringType
    return isinstance(field.dataType, StringType)


def is_bytes_field(field) -> bool:
    """String or binary schema field: shuffled as tensors (shuffle_strings)."""
    from ..frame.types import BinaryType, StringType
    return isinstance(field.dataType, (StringType, BinaryType))


def shuffle_strings(per_dest: List[Any], recv_rows: List[int], binary: bool):
    """String / binary column rows per destination rank -> the rows this rank
    receives (source-rank order), as one StringColumn. Moves an int64 length
    tensor and a uint8 byte tensor in two all_to_alls: no Python object per
    row crosses a rank (reference counterpart: the groupBy / repartition
    shuffle, DebugRowOps.scala:576)."""
    from ..frame.block import StringColumn, concat_columns
    from ..ops import groupby as G
    cols = [G.as_string_column(c, binary).to(torch.device("cpu")) if c is not None and len(c)
            else StringColumn.from_values([], binary) for c in per_dest]
    cat = concat_columns(cols) if len(cols) > 1 else cols[0]
    lens = cat.lengths().contiguous()
    got_lens = dist.all_to_all_rows(lens, [len(c) for c in cols], [int(r) for r in recv_rows])
    send_b = [int(c.data.numel()) for c in cols]
    # what each source sends us, in bytes: the sums of its received lengths
    recv_b, off = [], 0
    for r in recv_rows:
        recv_b.append(int(got_lens[off:off + int(r)].sum()) if int(r) else 0)
        off += int(r)
    got = dist.all_to_all_rows(cat.data.contiguous(), send_b, recv_b)
    offs = torch.zeros(got_lens.shape[0] + 1, dtype=torch.int64)
    torch.cumsum(got_lens, 0, out=offs[1:])
    return StringColumn(offs, got, binary)


def _gather_strings(local, owned, counts, rows_of_rank, root, w) -> Optional[Dict[int, List[str]]]:
    """String column of every partition (in pid order) as value lists, moved
    as an int64 length tensor and a uint8 byte tensor per rank."""
    from ..frame.block import StringColumn, concat_columns
    from ..ops import groupby as G
    cols = [G.as_string_column(c).to(torch.device("cpu")) for _, c in sorted(local, key=lambda x: x[0])]
    cat = concat_columns(cols) if cols else StringColumn.from_values([])
    nb = torch.zeros(w, dtype=torch.int64)
    nb[dist.rank()] = int(cat.data.numel())
    dist.all_reduce_host_(nb, "Sum")
    lens = dist.gather_rows(cat.lengths().contiguous(), rows_of_rank, root)
    data = dist.gather_rows(cat.data.contiguous(), nb.tolist(), root)
    if lens is None:
        return None
    out: Dict[int, List[str]] = {}
    for r in range(w):
        ln = lens[r]
        offs = torch.zeros(ln.shape[0] + 1, dtype=torch.int64)
        torch.cumsum(ln, 0, out=offs[1:])
        sc = StringColumn(offs, data[r])
        a = 0
        for p in owned[r]:
            out[p] = sc.slice(a, a + counts[p]).values
            a += counts[p]
    return out


def gather_blocks(local: List[Tuple[int, Any]], names: Sequence[str], schema, nparts: int,
                  root: Optional[int] = None) -> Optional[List[Tuple[int, int, List[Any]]]]:
    """[(pid, nrows, [column payload per name])] of EVERY partition, in pid
    order, on every rank (root None) or on `root` only (None elsewhere).
    Payloads: numpy arrays [rows, *cell] for dense columns, value lists
    otherwise."""
    from ..frame.block import column_values
    w, me = dist.world_size(), dist.rank()
    counts = partition_rows({p: b.nrows for p, b in local}, nparts)
    owned = {r: [p for p in range(nparts) if p % w == r] for r in range(w)}
    rows_of_rank = [sum(counts[p] for p in owned[r]) for r in range(w)]
    kinds = column_kinds([b for _, b in local], names, schema)
    local = sorted(local)
    per_col: Dict[str, Dict[int, Any]] = {}
    for n in names:
        k = kinds[n]
        if k is not None:
            mine = _host_cat([b.columns[n] for _, b in local if b.nrows], k)
            got = dist.gather_rows(mine, rows_of_rank, root)
            if got is None:
                continue
            byp: Dict[int, Any] = {}
            for r in range(w):
                a, arr = 0, got[r].numpy()
                for p in owned[r]:
                    byp[p] = arr[a:a + counts[p]]
                    a += counts[p]
            per_col[n] = byp
        elif _is_string_field(schema[n]):
            # strings as two tensors (lengths + bytes), no pickling
            per_col[n] = _gather_strings([(p, b.columns[n]) for p, b in local if b.nrows], owned, counts,
                                         rows_of_rank, root, w)
            if per_col[n] is None:
                del per_col[n]
        else:
            mine = [(p, column_values(b.columns[n])) for p, b in local if b.nrows]
            got = dist.all_gather_object(mine) if root is None else dist.gather_object(mine, root)
            if got is None:
                continue
            per_col[n] = {p: v for chunk in got for p, v in chunk}
    if root is not None and me != root:
        return None
    return [(p, counts[p], [per_col[n][p] for n in names]) for p in range(nparts) if counts[p]]


def take_rows(it, names: Sequence[str], schema, nparts: int, n: int) -> List[Tuple[int, List[Any]]]:
    """The first n rows in partition order as [(nrows, payloads)] on every
    rank: partitions are evaluated in order until n rows are in hand (later
    ones are never computed) and each partition's owner broadcasts only the
    rows still needed, dense columns as tensors."""
    from ..frame.block import column_values
    w = dist.world_size()
    local_iter = iter(it)
    buffered: Dict[int, Any] = {}
    kinds: Optional[Dict[str, Kind]] = None

    def local_block(p: int):
        while p not in buffered:
            try:
                pid, b = next(local_iter)
            except StopIteration:
                return None
            buffered[pid] = b
        return buffered.pop(p)

    out: List[Tuple[int, List[Any]]] = []
    got = 0
    for p in range(nparts):
        need = n - got
        owner = p % w if dist.is_distributed() else 0
        b = local_block(p) if owner == dist.rank() else None
        k = min(need, b.nrows) if b is not None else 0
        if dist.is_distributed():
            kt = dist.broadcast_tensor(torch.tensor([k], dtype=torch.int64), (1,), torch.int64, owner)
            k = int(kt.item())
            if kinds is None:
                # decided from the schema (plus a tiny exchange for columns it does not pin)
                kinds = column_kinds([b] if b is not None else [], names, schema)
        if k:
            cols = []
            for c in names:
                kind = kinds.get(c) if kinds is not None else None
                if not dist.is_distributed():
                    col = b.columns[c]
                    cols.append(col[:k].detach().cpu().numpy() if isinstance(col, torch.Tensor)
                                else column_values(col)[:k])
                elif kind is not None:
                    src = b.columns[c][:k].detach().cpu() if b is not None else None
                    cols.append(dist.broadcast_tensor(src, (k,) + kind[1], kind[0], owner).numpy())
                else:
                    vals = column_values(b.columns[c])[:k] if b is not None else None
                    cols.append(dist.broadcast_object(vals, src=owner))
            out.append((k, cols))
            got += k
        if got >= n:
            break
    return out


def _agreed_devices(local: Dict[int, Any], names: Sequence[str]) -> Dict[str, torch.device]:
    """Where each dense column's all-to-all runs, the SAME on every rank: the
    GPU (RCCL) only when every rank that holds rows of it holds them on the
    device. A rank with no local rows (more ranks than partitions, or empty
    partitions) follows the others instead of deciding from nothing, so the
    ranks never issue mismatched collectives (RCCL on some, gloo on others).
    One small Min all-reduce for all columns."""
    from .. import engine
    if not names:
        return {}
    gpu_ok = dist.is_distributed() and dist.gpu_collectives() and engine.gpu_available()
    flags = []
    for n in names:
        srcs = [local[p].columns[n] for p in local if local[p].nrows]
        # 1 = "device is fine with me"; a rank without rows abstains (1), and
        # an all-abstaining column (no rows anywhere) stays on the host (has)
        flags.append([int(all(c.is_cuda for c in srcs)), -int(bool(srcs))])
    t = torch.tensor(flags, dtype=torch.int64).reshape(-1)
    dist.all_reduce_host_(t, "Min")
    t = t.reshape(len(names), 2)
    out = {}
    for i, n in enumerate(names):
        on_gpu = gpu_ok and bool(t[i, 0]) and int(t[i, 1]) < 0
        out[n] = engine.compute_device() if on_gpu else torch.device("cpu")
    return out


def repartition_blocks(local: Dict[int, Any], names: Sequence[str], schema, nparts_in: int,
                       nparts_out: int) -> Dict[int, Any]:
    """Rows re-sliced into nparts_out even partitions (in row order); each
    rank receives only the rows of the partitions it owns: dense columns in
    one all-to-all per column (RCCL for device-resident frames), other
    columns as pickled values."""
    from ..frame.block import Block, build_column, column_tf_dtype, column_values
    from .. import engine
    w, me = dist.world_size(), dist.rank()
    counts = partition_rows({p: b.nrows for p, b in local.items()}, nparts_in)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    total = int(offs[-1])
    qb = [(q * total) // nparts_out for q in range(nparts_out + 1)]

    def pieces_of(p: int):
        """(q, start within p, length) of the new partitions overlapping p."""
        a0, a1 = int(offs[p]), int(offs[p + 1])
        res = []
        for q in range(nparts_out):
            lo, hi = max(a0, qb[q]), min(a1, qb[q + 1])
            if hi > lo:
                res.append((q, lo - a0, hi - lo))
        return res

    # what this rank sends to each rank r, ordered by (q, p)
    send: List[List[Tuple[int, int, int, int]]] = [[] for _ in range(w)]  # (q, p, start, len)
    for p in sorted(local):
        for q, st, ln in pieces_of(p):
            send[q % w].append((q, p, st, ln))
    for r in range(w):
        send[r].sort()
    # what this rank receives from each source rank s, in s's send order
    recv: List[List[Tuple[int, int, int, int]]] = [[] for _ in range(w)]
    for p in range(nparts_in):
        for q, st, ln in pieces_of(p):
            if q % w == me:
                recv[p % w].append((q, p, st, ln))
    for s in range(w):
        recv[s].sort()
    send_rows = [sum(x[3] for x in send[r]) for r in range(w)]
    recv_rows = [sum(x[3] for x in recv[s]) for s in range(w)]
    kinds = column_kinds(list(local.values()), names, schema)
    mine = [q for q in range(nparts_out) if q % w == me]
    cols_out: Dict[int, Dict[str, Any]] = {q: {} for q in mine}
    devs = _agreed_devices(local, [n for n in names if kinds[n] is not None])
    for n in names:
        kind = kinds[n]
        if kind is not None:
            dev = devs[n]
            parts = [local[p].columns[n][st:st + ln].to(dev) for r in range(w) for (_, p, st, ln) in send[r]]
            buf = engine.cat_rows(parts) if parts else engine.device_empty((0,) + kind[1], kind[0], dev)
            got = dist.all_to_all_rows(buf, send_rows, recv_rows) if dist.is_distributed() else buf
            pos, pieces = 0, {q: [] for q in mine}
            for s in range(w):
                for (q, p, st, ln) in recv[s]:
                    pieces[q].append((p, got[pos:pos + ln]))
                    pos += ln
            for q in mine:
                ps = [t for _, t in sorted(pieces[q], key=lambda x: x[0])]
                cols_out[q][n] = engine.cat_rows(ps) if ps else engine.device_empty((0,) + kind[1], kind[0], dev)
        elif is_bytes_field(schema[n]) and dist.is_distributed():
            from ..frame.block import concat_columns
            from ..frame.types import BinaryType
            from ..ops import groupby as G
            binary = isinstance(schema[n].dataType, BinaryType)
            per_dest = []
            for r in range(w):
                ps = [G.as_string_column(local[p].columns[n], binary).slice(st, st + ln) for (_, p, st, ln) in send[r]]
                per_dest.append(concat_columns(ps) if ps else None)
            got = shuffle_strings(per_dest, recv_rows, binary)
            pos, pieces = 0, {q: [] for q in mine}
            for s_ in range(w):
                for (q, p, st, ln) in recv[s_]:
                    pieces[q].append((p, got.slice(pos, pos + ln)))
                    pos += ln
            for q in mine:
                ps = [c for _, c in sorted(pieces[q], key=lambda x: x[0])]
                cols_out[q][n] = concat_columns(ps) if ps else _empty_strings(binary)
        else:
            tfd = _schema_tf(schema[n])
            if tfd is None:
                tfd = next((column_tf_dtype(local[p].columns[n]) for p in local), None)
            payload = [[column_values(local[p].columns[n])[st:st + ln] for (_, p, st, ln) in send[r]]
                       for r in range(w)]
            got = dist.all_to_all_objects(payload) if dist.is_distributed() else payload
            pieces = {q: [] for q in mine}
            for s in range(w):
                for (q, p, st, ln), vals in zip(recv[s], got[s]):
                    pieces[q].append((p, vals))
            for q in mine:
                vals = [v for _, vs in sorted(pieces[q], key=lambda x: x[0]) for v in vs]
                cols_out[q][n] = build_column(vals, tfd)
    return {q: Block(qb[q + 1] - qb[q], cols_out[q]) for q in mine}

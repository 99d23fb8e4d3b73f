"""groupBy segmentation and the keyed shuffle, on the device.

Keys of a block are factorised where they live: on a GPU by the radix-sort
kernels of csrc/kernels/groupby.hip (`_C.factorize`), on the host by the ATen
oracle. Groups come out in ascending key order (lexicographic for several
key columns), the order the reference's Spark groupBy results are compared in
(reference: src/test/scala/org/tensorframes/BasicOperationsSuite.scala:200-210
via compareRows). String keys never become Python objects: their bytes are
packed into big-endian 64-bit words + a length (`_C.string_words`), which the
same numeric kernels group exactly and in lexicographic order.

The cross-rank shuffle of per-key partials hashes the keys on the device
(`_C.key_dest`: the same 64-bit hash on every rank), orders the rows by
destination with one radix sort (`_C.partition_rows`), packs every column of
a row into one record in that order (`_C.pack_rows`) and exchanges the
records in ONE all-to-all (RCCL for device tensors), unpacked on arrival. Reference counterpart: the UDAF shuffle
(src/main/scala/org/tensorframes/impl/DebugRowOps.scala:573-576).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from .._native import _C
from ..parallel import dist

_KEY_DTYPES = (torch.float32, torch.float64, torch.int32, torch.int64)


def device_keys(cols: Sequence) -> bool:
    """All key columns are dense 1-D numeric tensors the kernels can factorise."""
    return all(isinstance(c, torch.Tensor) and c.dim() == 1 and c.dtype in _KEY_DTYPES for c in cols)


def group_ids(keys: List[torch.Tensor]) -> Tuple[torch.Tensor, List[torch.Tensor], int]:
    """(group id of every row [n] int64, distinct key columns [ngroups], ngroups).

    One key: a single factorisation. Several keys: each column is factorised,
    the codes are combined lexicographically (code * n_next + id_next) and
    re-factorised after every column, so codes stay below n and the group
    order stays lexicographic; the key values of each group are read from one
    representative row."""
    n = keys[0].shape[0]
    if n == 0:
        return (torch.empty(0, dtype=torch.int64, device=keys[0].device),
                [k[:0] for k in keys], 0)
    if len(keys) == 1:
        ids, uniq = _C.factorize(keys[0])
        return ids, [uniq], int(uniq.shape[0])
    code, _ = _C.factorize(keys[0])
    for k in keys[1:]:
        ids_k, uniq_k = _C.factorize(k)
        code, _ = _C.factorize(code * int(uniq_k.shape[0]) + ids_k)
    ids, ucode = _C.factorize(code)
    ng = int(ucode.shape[0])
    if ids.is_cuda:
        rep = _C.group_representatives(ids, ng)
        uniq = [_C.gather_rows(k.contiguous(), rep) for k in keys]
    else:
        rep = torch.empty(ng, dtype=torch.int64)
        rep[ids] = torch.arange(n, dtype=torch.int64)
        uniq = [k[rep] for k in keys]
    return ids, uniq, ng


def route(keys: List[torch.Tensor], cols: List[torch.Tensor]) -> List[torch.Tensor]:
    """Keyed all-to-all: rows go to rank hash(keys) % world; returns the
    received columns (keys first, then `cols`), concatenated in source-rank
    order. Device columns: hash, partition and gather on the GPU, exchange
    over RCCL; every rank takes part even with no rows."""
    w = dist.world_size()
    allc = list(keys) + list(cols)
    dev = allc[0].device
    n = allc[0].shape[0]
    if dev.type == "cuda" and len(allc) <= 16:
        # every column of a row packed into one record: the rows move in ONE
        # all-to-all (plus the tiny count exchange), not one per column
        dest = _C.key_dest([k.contiguous() for k in keys], w) if n else torch.empty(0, dtype=torch.int64, device=dev)
        perm, counts = _C.partition_rows(dest, w)
        send_rows = [int(c) for c in counts.cpu().tolist()]
        recv_rows = dist.all_to_all_counts(send_rows)
        rec, _ = _C.pack_rows([c.contiguous() for c in allc], perm)
        got = dist.all_to_all_rows(rec, send_rows, recv_rows)
        m = int(sum(recv_rows))
        outs = [torch.empty((m,) + tuple(c.shape[1:]), dtype=c.dtype, device=dev) for c in allc]
        if m:
            _C.unpack_rows(got, outs)
        return outs
    if dev.type == "cuda":
        dest = _C.key_dest([k.contiguous() for k in keys], w) if n else torch.empty(0, dtype=torch.int64, device=dev)
        perm, counts = _C.partition_rows(dest, w)
        send_rows = [int(c) for c in counts.cpu().tolist()]
        ordered = [_C.gather_rows(c.contiguous(), perm) if n else c for c in allc]
    else:
        from ..core import _key_hash
        dest = (_key_hash([k.numpy() for k in keys]) % np.uint64(w)).astype(np.int64) if n else np.zeros(0, np.int64)
        perm = torch.from_numpy(np.argsort(dest, kind="stable"))
        send_rows = np.bincount(dest, minlength=w).tolist()
        ordered = [c[perm] for c in allc]
    recv_rows = dist.all_to_all_counts(send_rows)
    return [dist.all_to_all_rows(c, send_rows, recv_rows) for c in ordered]


# ---------------------------------------------------------------- string keys
def as_string_column(col, binary: bool = False):
    """A key column of str / bytes values as an Arrow-layout StringColumn."""
    from ..frame.block import StringColumn
    if isinstance(col, StringColumn):
        return col
    return StringColumn.from_values(list(col.values), binary)


def string_width(cols: Sequence) -> int:
    """Words (8 bytes each) that hold the longest string of these columns, >= 1."""
    longest = 0
    for c in cols:
        if len(c):
            longest = max(longest, int(c.lengths().max()))
    return max(1, -(-longest // 8))


def string_key_words(col, words: int, dev: torch.device) -> List[torch.Tensor]:
    """[word 0, ..., word W-1, length] int64 key columns of one string column
    on `dev` (kernels/groupby.hip string_words): grouped by the numeric
    factorisation they sort lexicographically and compare exactly."""
    col = col.to(dev)
    packed = _C.string_words(col.offsets, col.data, int(words))  # [W + 1, n]
    return [packed[j] for j in range(words + 1)]


def words_to_strings(cols: List[torch.Tensor], binary: bool = False):
    """Inverse of string_key_words for the (few) group keys: -> StringColumn (host)."""
    from ..frame.block import StringColumn
    w = len(cols) - 1
    lens = cols[w].cpu().numpy().astype(np.int64)
    n = len(lens)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    if n == 0:
        return StringColumn(torch.from_numpy(offs), torch.zeros(0, dtype=torch.uint8), binary)
    words = torch.stack([c.cpu() for c in cols[:w]], 1).numpy()  # [n, W]
    u = (words.view(np.uint64) ^ np.uint64(1 << 63)).astype(">u8")
    raw = u.view(np.uint8).reshape(n, 8 * w)
    mask = np.arange(8 * w)[None, :] < lens[:, None]
    return StringColumn(torch.from_numpy(offs), torch.from_numpy(np.ascontiguousarray(raw[mask])), binary)

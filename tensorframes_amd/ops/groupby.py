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

from typing import List, Optional, Sequence, Tuple

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
        return (engine_empty(0, torch.int64, keys[0].device),
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


def route(keys: List[torch.Tensor], cols: List[torch.Tensor], strings: Optional[Sequence] = None):
    """Keyed all-to-all: rows go to rank hash(keys) % world; returns the
    received columns (keys first, then `cols`), concatenated in source-rank
    order. With `strings` (string columns row-aligned with the keys: the
    hashed string keys' strings, host or device) returns (columns, their
    received rows as host StringColumns; lengths + bytes move in two
    all-to-alls, frame_comm.shuffle_strings). Device columns: hash,
    partition and gather on the GPU, exchange over RCCL; every rank takes
    part even with no rows."""
    w = dist.world_size()
    allc = list(keys) + list(cols)
    dev = allc[0].device
    n = allc[0].shape[0]
    if dev.type == "cuda":
        dest = _C.key_dest([k.contiguous() for k in keys], w) if n else engine_empty(0, torch.int64, dev)
        perm, counts = _C.partition_rows(dest, w)
        send_rows = [int(c) for c in counts.cpu().tolist()]
    else:
        from ..core import _key_hash
        dest = (_key_hash([k.numpy() for k in keys]) % np.uint64(w)).astype(np.int64) if n else np.zeros(0, np.int64)
        perm = torch.from_numpy(np.argsort(dest, kind="stable"))
        send_rows = np.bincount(dest, minlength=w).tolist()
    recv_rows = dist.all_to_all_counts(send_rows)
    if dev.type == "cuda" and len(allc) <= 16:
        # every column of a row packed into one record: the rows move in ONE
        # all-to-all (plus the tiny count exchange), not one per column
        rec, _ = _C.pack_rows([c.contiguous() for c in allc], perm)
        got = dist.all_to_all_rows(rec, send_rows, recv_rows)
        m = int(sum(recv_rows))
        outs = [engine_empty((m,) + tuple(c.shape[1:]), c.dtype, dev) for c in allc]
        if m:
            _C.unpack_rows(got, outs)
    else:
        if dev.type == "cuda":
            ordered = [_C.gather_rows(c.contiguous(), perm) if n else c for c in allc]
        else:
            ordered = [c[perm] for c in allc]
        outs = [dist.all_to_all_rows(c, send_rows, recv_rows) for c in ordered]
    if strings is None:
        return outs
    from ..parallel import frame_comm
    bounds = np.concatenate([[0], np.cumsum(send_rows)]).astype(np.int64)
    got_s = []
    for sc in strings:
        srt = gather_strings(sc, perm) if len(sc) else sc.to(torch.device("cpu"))
        per = [srt.slice(int(bounds[r]), int(bounds[r + 1])) for r in range(w)]
        got_s.append(frame_comm.shuffle_strings(per, recv_rows, sc.binary))
    return outs, got_s


def engine_empty(shape, dtype, dev):
    from .. import engine
    return engine.device_empty(shape, dtype, dev)


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


# ------------------------------------------------ bounded-width string keys
class StringKeyCollision(RuntimeError):
    """Two different string keys shared (word 0, tag)."""


HASH_TAG_MIN = 9  # tags >= 9 are hashed long keys (tag = length below)


def string_key_hashed(col, dev: torch.device) -> List[torch.Tensor]:
    """[word 0, tag] int64 key columns (kernels/groupby.hip string_key_hash):
    2 words per row whatever the longest key. Keys of <= 8 bytes are exact
    (tag = length); longer ones carry tag = 9 + a 62-bit hash of all their
    bytes, verified against one representative per group (group_keys)."""
    col = col.to(dev)
    packed = _C.string_key_hash(col.offsets, col.data)
    return [packed[0], packed[1]]


def concat_strings(cols: Sequence):
    """One StringColumn of these (same device; device buffers from the pool)."""
    from .. import engine
    from ..frame.block import StringColumn
    if len(cols) == 1:
        return cols[0]
    dev = cols[0].offsets.device
    n = sum(len(c) for c in cols)
    nbytes = sum(int(c.offsets[-1] - c.offsets[0]) for c in cols)
    offs = engine.device_empty(n + 1, torch.int64, dev)
    data = engine.device_empty(nbytes, torch.uint8, dev)
    offs[:1].copy_(torch.zeros(1, dtype=torch.int64))
    r = b = 0
    for c in cols:
        lo, hi, m = int(c.offsets[0]), int(c.offsets[-1]), len(c)
        torch.add(c.offsets[1:], b - lo, out=offs[r + 1:r + 1 + m])
        data[b:b + hi - lo].copy_(c.data[lo:hi])
        r, b = r + m, b + hi - lo
    return StringColumn(offs, data, cols[0].binary)


def gather_strings(col, idx: torch.Tensor):
    """Rows `idx` of a string column, as a host StringColumn (a device column
    is gathered on the device: only the selected bytes cross PCIe)."""
    from ..frame.block import StringColumn
    if col.is_cuda:
        offs, data = _C.gather_strings(col.offsets, col.data, idx.to(col.data.device))
        return StringColumn(offs, data.cpu(), col.binary)
    return col.take(idx.cpu().numpy())


def representatives(ids: torch.Tensor, ng: int) -> torch.Tensor:
    """One row index per group (device ids: on the device)."""
    if ids.is_cuda:
        return _C.group_representatives(ids, ng)
    rep = np.empty(ng, dtype=np.int64)
    rep[ids.numpy()] = np.arange(ids.shape[0], dtype=np.int64)
    return torch.from_numpy(rep)


def _tie_runs(uniq: List[np.ndarray], p: int) -> np.ndarray:
    """Adjacent group pairs equal on every expanded column up to p (the hashed
    key's word 0) whose keys are both long (hash >= 1): their relative order
    is the hash's, not the strings'."""
    same = np.ones(len(uniq[0]) - 1, dtype=bool)
    for c in uniq[:p + 1]:
        eq = c[1:] == c[:-1]
        if c.dtype.kind == "f":
            eq |= np.isnan(c[1:]) & np.isnan(c[:-1])
        same &= eq
    t = uniq[p + 1]
    return same & (t[1:] >= HASH_TAG_MIN) & (t[:-1] >= HASH_TAG_MIN)


def exact_hashed_order(uniq: List[torch.Tensor], ustr: dict) -> Optional[np.ndarray]:
    """Group order fix for hashed string keys. Groups come out sorted by
    (word 0, tag, ...): exact except among long keys sharing their
    first 8 bytes, which sort by hash. Within each such run the groups are
    re-sorted (stably) by their exact bytes; groups of equal strings are
    already contiguous and ordered by the later key columns. Returns the new
    group order, or None when no run exists (the common case)."""
    ng = int(uniq[0].shape[0])
    if ng < 2 or not ustr:
        return None
    perm = None
    for p in sorted(ustr):
        cols = [u.cpu().numpy() for u in uniq[:p + 2]]
        if perm is not None:
            cols = [c[perm] for c in cols]
        ties = _tie_runs(cols, p)
        if not ties.any():
            continue
        vals = ustr[p].values
        if perm is None:
            perm = np.arange(ng, dtype=np.int64)
        raw = [v if isinstance(v, (bytes, bytearray)) else v.encode("utf-8") for v in vals]
        i = 0
        while i < ng - 1:
            if not ties[i]:
                i += 1
                continue
            j = i
            while j < ng - 1 and ties[j]:
                j += 1
            run = perm[i:j + 1]
            perm[i:j + 1] = np.asarray(sorted(run.tolist(), key=lambda g: raw[g]), dtype=np.int64)
            i = j + 1
    return perm


def group_keys(K: List[torch.Tensor], hashed: dict):
    """group_ids + the hashed string keys' checks. hashed: {position of the
    key's word-0 column in K: StringColumn of the rows}. Returns (ids, uniq
    columns, ngroups, {position: StringColumn of the group keys, host}).
    Raises StringKeyCollision when a group holds two different strings."""
    ids, uniq, ng = group_ids(K)
    if not hashed or ng == 0:
        return ids, uniq, ng, {p: gather_strings(s, ids[:0]) for p, s in hashed.items()}
    rep = representatives(ids, ng)
    ustr = {}
    for p, sc in hashed.items():
        if not _C.string_verify(sc.offsets, sc.data, ids.to(sc.data.device), rep.to(sc.data.device)):
            raise StringKeyCollision("string keys: two different keys share (8-byte prefix, 62-bit hash)")
        ustr[p] = gather_strings(sc, rep)
    perm = exact_hashed_order(uniq, ustr)
    if perm is not None:
        inv = np.empty_like(perm)
        inv[perm] = np.arange(ng, dtype=np.int64)
        inv_t = torch.from_numpy(inv).to(ids.device)
        perm_t = torch.from_numpy(perm).to(ids.device)
        if ids.is_cuda:
            ids = _C.gather_rows(inv_t, ids)
            uniq = [_C.gather_rows(u.contiguous(), perm_t) for u in uniq]
        else:
            ids = inv_t[ids]
            uniq = [u[perm_t] for u in uniq]
        ustr = {p: s.take(perm) for p, s in ustr.items()}
    return ids, uniq, ng, ustr

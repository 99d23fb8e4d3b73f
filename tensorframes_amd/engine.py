"""Execution engine: compiled programs, device placement, host<->device staging.

One `Program` (native: csrc/runtime/executor.*) per (graph, fetches, feeds)
is cached and shared by every partition and every call, so a graph is parsed,
shape-inferred and planned once and its constants are uploaded to HBM once —
the reference instead imports the GraphDef into a fresh TF session per
partition (reference: src/main/scala/org/tensorframes/impl/DebugRowOps.scala:766-803,
src/main/scala/org/tensorframes/impl/TensorFlowOps.scala:76-95).

Block execution on a GPU:
  * device-resident blocks run in place;
  * large host blocks of a row-separable graph stream through a pipelined
    chunk loop (pinned host -> HBM on a copy stream, kernels on the compute
    stream, HBM -> pinned host on a second copy stream);
  * anything else: one H2D, run, one D2H.
"""
from __future__ import annotations

import hashlib
import os
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._native import _C
from .config import config
from .parallel import dist
from .utils import dtypes as D
from .utils.logging import logger, metrics

_graph_cache: "OrderedDict[str, object]" = OrderedDict()
_prog_cache: "OrderedDict[tuple, object]" = OrderedDict()
_lock = threading.Lock()
_MAX_CACHE = 64


_hash_memo: "OrderedDict[int, Tuple[bytes, str]]" = OrderedDict()
_graph_bytes_cached = 0
_MAX_GRAPH_BYTES = 8 << 30  # native graphs kept alive (model weights live in them)


def _key(graph_bytes: bytes) -> str:
    """Content hash of a GraphDef, memoised by object identity: the DSL hands
    out the same bytes object until the graph changes, so big models
    (hundreds of MB of weights) are hashed once, not per operator call."""
    ent = _hash_memo.get(id(graph_bytes))
    if ent is not None and ent[0] is graph_bytes:
        return ent[1]
    k = hashlib.sha1(graph_bytes).hexdigest()
    with _lock:
        _hash_memo[id(graph_bytes)] = (graph_bytes, k)
        while len(_hash_memo) > 4:
            _hash_memo.popitem(last=False)
    return k


def native_graph(graph_bytes: bytes):
    global _graph_bytes_cached
    k = _key(graph_bytes)
    with _lock:
        ent = _graph_cache.get(k)
        if ent is not None:
            _graph_cache.move_to_end(k)
            return ent[0]
    g = _C.Graph(graph_bytes)
    with _lock:
        _graph_cache[k] = (g, len(graph_bytes))
        _graph_bytes_cached += len(graph_bytes)
        while len(_graph_cache) > 1 and (len(_graph_cache) > _MAX_CACHE or _graph_bytes_cached > _MAX_GRAPH_BYTES):
            _, (_, nb) = _graph_cache.popitem(last=False)
            _graph_bytes_cached -= nb
    return g


_struct_cache: "OrderedDict[tuple, object]" = OrderedDict()


def structure_key(graph_bytes: bytes) -> int:
    """Graph::structure_key of the graph: equal for graphs that differ only
    in the payloads of parameter constants (e.g. K-Means centres)."""
    return native_graph(graph_bytes).structure_key()


def program(graph_bytes: bytes, fetches: Sequence[str], feeds: Sequence[str]):
    """The cached program for (graph, fetches, feeds). A new graph with the
    structure of an earlier one (only parameter constants changed: an
    iterative workload rebuilding its graph every step, reference
    kmeans_demo.py:101-168) takes over that program's plans, fused kernels,
    HIP-graph captures and constant arenas instead of planning again
    (executor.h Program::adopt); the earlier program stays usable."""
    k = (_key(graph_bytes), tuple(fetches), tuple(feeds))
    with _lock:
        p = _prog_cache.get(k)
        if p is not None:
            _prog_cache.move_to_end(k)
            return p
    g = native_graph(_planned_bytes(graph_bytes))
    p = _C.Program(g, list(fetches), list(feeds))
    if config.plan_reuse:
        sk = (g.structure_key(), tuple(fetches), tuple(feeds))
        with _lock:
            old = _struct_cache.get(sk)
        if old is not None and p.adopt(old):
            metrics.add("programs_adopted")
        with _lock:
            _struct_cache[sk] = p
            _struct_cache.move_to_end(sk)
            while len(_struct_cache) > _MAX_CACHE:
                _struct_cache.popitem(last=False)
    with _lock:
        _prog_cache[k] = p
        while len(_prog_cache) > _MAX_CACHE:
            _prog_cache.popitem(last=False)
    return p


# (Graph.fast_key structure, fetches, feeds) -> [program, parameter names,
# payloads of the other float constants, payloads the program was built with]
_fast_progs: "OrderedDict[tuple, list]" = OrderedDict()


def program_for_spec(spec, fetches: Sequence[str], feeds: Sequence[str]):
    """`program(spec.graph_bytes, fetches, feeds)` for a resolved graph. A DSL
    graph whose structure (Graph.fast_key: everything but the payloads of its
    floating constants) is known gets the known program with the new
    parameter payloads swapped in (Program.rebind: plans, fused kernels and
    HIP-graph captures carried over) -- no serialisation, hash or parse of the
    rebuilt graph (an iterative workload: reference kmeans_demo.py:101-168)."""
    fk = spec.fast_key()
    if fk is None:
        return program(spec.graph_bytes, fetches, feeds)
    skey, params = fk
    k = (skey, tuple(fetches), tuple(feeds))
    with _lock:
        ent = _fast_progs.get(k)
        if ent is not None:
            _fast_progs.move_to_end(k)
    if ent is not None:
        prog, pnames, fixed, built = ent
        if all(params[n].content == b for n, b in fixed.items()):
            if all(params[n].content == built[n] for n in pnames):
                return prog  # the same payloads: the same program
            vals = {n: _tensor_of(params[n]) for n in pnames}
            p = prog.rebind(vals)
            metrics.add("programs_rebound")
            with _lock:
                _fast_progs[k] = [p, pnames, fixed, {n: params[n].content for n in pnames}]
            return p
    gb = spec.graph_bytes
    p = program(gb, fetches, feeds)
    if _planned_bytes(gb) is gb:  # no rewrite changed the graph: its constants are the user's
        pnames = set(native_graph(gb).parameter_consts()) & set(params)
        with _lock:
            _fast_progs[k] = [p, pnames, {n: tp.content for n, tp in params.items() if n not in pnames},
                              {n: params[n].content for n in pnames}]
            while len(_fast_progs) > _MAX_CACHE:
                _fast_progs.popitem(last=False)
    return p


def _tensor_of(tp) -> torch.Tensor:
    from .utils import dtypes as D
    npdt = np.dtype(D.numpy_dtype(tp.dtype)).newbyteorder("<")
    return torch.from_numpy(np.frombuffer(tp.content, dtype=npdt).reshape(tp.shape).copy())


_rewritten: "OrderedDict[str, bytes]" = OrderedDict()


def _planned_bytes(graph_bytes: bytes) -> bytes:
    """The GraphDef the executor plans: the user's, after the algebraic
    rewrites of graph/rewrite.py (value-preserving for every fetch;
    `Config.graph_rewrites` = False plans the graph as given)."""
    if not config.graph_rewrites:
        return graph_bytes
    k = _key(graph_bytes)
    with _lock:
        if k in _rewritten:
            return _rewritten[k] or graph_bytes
    from .graph import rewrite
    out = rewrite.optimize(graph_bytes)
    with _lock:
        _rewritten[k] = out
        while len(_rewritten) > _MAX_CACHE:
            _rewritten.popitem(last=False)
    return out or graph_bytes


def clear_program_cache():
    with _lock:
        _prog_cache.clear()
        _struct_cache.clear()
        _fast_progs.clear()
    from . import core  # memoised operator setups hold programs too
    core._REDUCE_SETUP.clear()


# ------------------------------------------------------------------ devices
_cuda_ok: Optional[bool] = None
_dev_memo: Dict[Tuple[str, str], torch.device] = {}


def gpu_available() -> bool:
    # torch.cuda.is_available() asks the runtime each time (~2 us; an
    # iterative workload asked it 17 times per step): whether this process
    # sees a GPU does not change, so it is asked once
    global _cuda_ok
    if config.device == "cpu":
        return False
    if _cuda_ok is None:
        _cuda_ok = torch.cuda.is_available()
    return _cuda_ok


def compute_device() -> torch.device:
    if gpu_available():
        lr = os.environ.get("LOCAL_RANK", "")
        d = _dev_memo.get((config.device, lr)) if lr else None
        if d is None:
            n = torch.cuda.device_count()
            d = torch.device("cuda", dist.local_rank() % max(n, 1))
            if lr:  # (without LOCAL_RANK the rank comes from a group that may start later)
                _dev_memo[(config.device, lr)] = d
        return d
    if config.device == "cuda":
        raise RuntimeError("TFA_DEVICE=cuda but no GPU is visible")
    return torch.device("cpu")


def small_work_device() -> torch.device:
    """Where tiny host work (per-row folds, small map_rows cells) runs: the
    host executor, unless `Config.device == "cuda"` forces every op onto the
    GPU (e.g. the GPU run of the acceptance corpus)."""
    if config.device == "cuda":
        return compute_device()
    return torch.device("cpu")


def to_device(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    if t.device == dev:
        return t
    return t.to(dev, non_blocking=is_pinned(t))


def empty_host(shape, dtype: torch.dtype, pinned: bool) -> torch.Tensor:
    nbytes = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
    if pinned and gpu_available() and nbytes >= config.pinned_min_bytes:
        return _C.empty_pinned(list(shape), dtype)
    return torch.empty(tuple(shape), dtype=dtype)


def device_empty(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """Uninitialised tensor; on a GPU it comes from the engine's own
    stream-ordered pool (csrc/runtime/device_pool.cpp), ordered on the
    device's current stream, instead of the framework allocator."""
    device = torch.device(device)
    if isinstance(shape, int):
        shape = (shape,)
    if device.type != "cuda":
        return torch.empty(tuple(shape), dtype=dtype, device=device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _C.device_empty([int(d) for d in shape], dtype, idx)


def device_zeros(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """Zeroed tensor; on a GPU from the engine pool, cleared by hipMemsetAsync."""
    device = torch.device(device)
    if isinstance(shape, int):
        shape = (shape,)
    if device.type != "cuda":
        return torch.zeros(tuple(shape), dtype=dtype, device=device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _C.device_zeros([int(d) for d in shape], dtype, idx)


def device_full(shape, value, dtype: torch.dtype, device) -> torch.Tensor:
    """Constant tensor; on a GPU from the engine pool, filled by the native
    fill kernel (values a double holds exactly) or copied from the host
    (64-bit integers beyond 2^53, e.g. the int64 Min/Max identities)."""
    device = torch.device(device)
    if isinstance(shape, int):
        shape = (shape,)
    if device.type != "cuda":
        return torch.full(tuple(shape), value, dtype=dtype, device=device)
    t = device_empty(shape, dtype, device)
    if t.numel() == 0:
        return t
    if dtype.is_floating_point or dtype == torch.bool or abs(int(value)) <= (1 << 53):
        return _C.fill_(t, float(value))
    t.copy_(torch.full(tuple(shape), value, dtype=dtype))
    return t


def record_stream(t: torch.Tensor, stream) -> None:
    """`t` is also used on `stream`: its memory is not reused before the work
    queued there so far has finished. Works for engine-pool tensors (for
    which torch's Tensor.record_stream is a no-op: c10 did not allocate them)
    and for framework tensors alike."""
    if t.is_cuda:
        _C.record_stream(t, int(stream.cuda_stream))


def cat_rows_many(cols: Sequence[Sequence[torch.Tensor]]) -> List[torch.Tensor]:
    """`[cat_rows(c) for c in cols]` for device columns, in one pool buffer
    and one batched-copy launch (the merged partitions of reduce_blocks: one
    launch instead of one per column)."""
    cols = [list(c) for c in cols]
    if (cols and all(c and c[0].is_cuda and c[0].dim() >= 1 for c in cols)
            and sum(len(c) for c in cols) <= 256
            and sum(t.numel() * t.element_size() for c in cols for t in c) <= (64 << 20)):
        return list(_C.cat_rows_many(cols))
    return [cat_rows(c) for c in cols]


def cat_rows(ts: Sequence[torch.Tensor]) -> torch.Tensor:
    """Concatenate along dim 0. Device tensors are copied into one pool
    buffer with device-to-device DMA (hipMemcpyAsync: contiguous same-dtype
    copy_), so no ATen concat kernel runs on the engine's GPU paths."""
    ts = list(ts)
    if len(ts) == 1:
        return ts[0]
    t0 = ts[0]
    if not t0.is_cuda:
        return torch.cat(ts, 0)
    if t0.dim() >= 1 and len(ts) <= 256 and sum(t.numel() * t.element_size() for t in ts) <= (64 << 20):
        # many small pieces (per-partition partials): one batched-copy kernel
        return _C.cat_rows(ts)
    out = device_empty((sum(int(t.shape[0]) for t in ts),) + tuple(t0.shape[1:]), t0.dtype, t0.device)
    a = 0
    for t in ts:
        b = a + int(t.shape[0])
        if b > a:
            out[a:b].copy_(t if t.is_contiguous() else t.contiguous())
        a = b
    return out


def stack_rows(ts: Sequence[torch.Tensor]) -> torch.Tensor:
    """torch.stack along a new dim 0, through cat_rows."""
    return cat_rows([t.unsqueeze(0) for t in ts])


def is_pinned(t: torch.Tensor) -> bool:
    return (not t.is_cuda) and gpu_available() and (t.is_pinned() or _C.is_pinned(t))


def pin(t: torch.Tensor) -> torch.Tensor:
    """Page-lock a host tensor for DMA (copy into pinned memory)."""
    if not gpu_available() or t.is_cuda or is_pinned(t):
        return t
    out = _C.empty_pinned(list(t.shape), t.dtype)
    out.copy_(t)
    return out


# ------------------------------------------------------------------ execution
def run_program(prog, inputs: List[torch.Tensor], dev: Optional[torch.device] = None) -> List[torch.Tensor]:
    """Run on one device; inputs are moved there if needed. Outputs stay on `dev`."""
    dev = dev or compute_device()
    ins = [to_device(t.contiguous(), dev) for t in inputs]
    if dev.type == "cuda":
        if dev.index is None or dev.index == torch.cuda.current_device():
            return list(prog.run(ins))  # (Program::run guards the inputs' device itself)
        with torch.cuda.device(dev):
            return list(prog.run(ins))
    if sum(t.numel() for t in ins) < config.cpu_parallel_min_elems:
        with _single_threaded():
            return list(prog.run(ins))
    return list(prog.run(ins))


_side_streams: Dict[int, List[torch.cuda.Stream]] = {}


def run_programs_concurrent(prog, inputs_list: List[List[torch.Tensor]], dev: torch.device,
                            max_streams: int = 4) -> List[List[torch.Tensor]]:
    """Several independent runs of one program (the device-resident partitions
    of a map_blocks) issued on up to 4 streams at once, so a GPU that one small
    partition cannot fill runs them side by side (K-Means: 4 partitions of
    25k rows, each a chain of small kernels). The results are ordered back
    onto the caller's stream before they are returned. The fork/join runs in
    C++ (Program::run_concurrent); the Python version below is the fallback
    for program objects without it."""
    if hasattr(prog, "run_concurrent"):
        # native fork/join (Program::run_concurrent): engine side streams,
        # events and pool-block bookkeeping in C++, GIL released
        ins_list = [[t.contiguous() for t in ins] for ins in inputs_list]
        if dev.index is None or dev.index == torch.cuda.current_device():
            outs = [list(o) for o in prog.run_concurrent(ins_list, max_streams)]
        else:
            with torch.cuda.device(dev):
                outs = [list(o) for o in prog.run_concurrent(ins_list, max_streams)]
        metrics.add("concurrent_partition_runs", len(inputs_list))
        return outs
    main = torch.cuda.current_stream(dev)
    pool = _side_streams.setdefault(dev.index, [])
    k = min(len(inputs_list), max_streams)
    while len(pool) < k:
        pool.append(torch.cuda.Stream(dev))
    ready = main.record_event()
    outs: List[List[torch.Tensor]] = []
    for i, ins in enumerate(inputs_list):
        st = pool[i % k]
        st.wait_event(ready)
        with torch.cuda.stream(st):
            outs.append(run_program(prog, ins, dev))
        for t in ins:
            record_stream(t, st)  # read on the side stream
    for st in pool[:k]:
        main.wait_stream(st)
    for o in outs:
        for t in o:
            if t.is_cuda:
                record_stream(t, main)  # side-stream memory, used on main from here on
    metrics.add("concurrent_partition_runs", len(inputs_list))
    return outs


_thread_lock = threading.Lock()


class _single_threaded:
    """Run small CPU programs on one intra-op thread: below a few million
    elements the OpenMP fork/join costs more than the op (tens of ms per op on
    virtualised hosts, measured)."""

    def __enter__(self):
        _thread_lock.acquire()
        self.n = torch.get_num_threads()
        if self.n != 1:
            torch.set_num_threads(1)

    def __exit__(self, *a):
        if self.n != 1:
            torch.set_num_threads(self.n)
        _thread_lock.release()


def worth_pipelining(inputs: List[torch.Tensor]) -> bool:
    """A host partition streams through the chunked H2D/compute/D2H pipeline
    when it has many rows or many bytes; smaller ones run in one shot."""
    if not inputs:
        return False
    rows = inputs[0].shape[0]
    nbytes = sum(t.numel() * t.element_size() for t in inputs)
    return rows >= 2 and (rows >= config.min_chunked_rows or nbytes >= config.min_chunked_bytes)


def run_block_host(prog, inputs: List[torch.Tensor], separable: bool,
                   out_specs: Optional[List[Tuple[tuple, torch.dtype]]] = None) -> List[torch.Tensor]:
    """Host-resident block -> host-resident outputs, on the compute device."""
    dev = compute_device()
    rows = inputs[0].shape[0] if inputs else 0
    if dev.type != "cuda":
        return [o.contiguous() for o in prog.run([t.contiguous() for t in inputs])]
    if separable and out_specs is not None and worth_pipelining(inputs):
        return run_segments_pipelined(prog, [inputs], [out_specs])[0]
    outs = run_program(prog, inputs, dev)
    res = []
    for o in outs:
        h = empty_host(tuple(o.shape), o.dtype, config.pinned_outputs)
        h.copy_(o, non_blocking=is_pinned(h))
        res.append(h)
    torch.cuda.current_stream(dev).synchronize()
    metrics.add("d2h_bytes", sum(o.numel() * o.element_size() for o in outs))
    return res


def chunk_rows_for(inputs: List[torch.Tensor], total_rows: Optional[int] = None) -> int:
    """Rows per pipelined chunk: at most `chunk_bytes` of the widest input,
    and small enough that a job yields >= `min_pipeline_chunks` chunks (a
    3-stage pipeline only overlaps once it has several chunks in flight),
    but not below 4 MB per DMA (or one row, for rows bigger than that:
    images)."""
    row_bytes = max((t[0].numel() * t.element_size() if t.shape[0] else 1) for t in inputs) if inputs else 1
    row_bytes = max(row_bytes, 1)
    rows = int(config.chunk_bytes // row_bytes)
    if total_rows:
        rows = min(rows, -(-total_rows // max(1, config.min_pipeline_chunks)))
    return max(1, (4 << 20) // row_bytes, rows)


_defer = threading.local()


class deferred_pipelines:
    """Inside this context, pipelined runs (run_segments_pipelined) return as
    soon as their copies and kernels are enqueued; their completions collect
    in the yielded list. A streaming action enqueues the next group of
    partitions before it waits for the previous one (wait_pipelines), so the
    chunk pipeline runs on across group boundaries (the next group's first H2D
    overlaps the previous group's last chunks) instead of draining and
    ramping up once per group."""

    def __enter__(self):
        self.prev = getattr(_defer, "handles", None)
        self.handles = []
        _defer.handles = self.handles
        return self.handles

    def __exit__(self, *exc):
        _defer.handles = self.prev
        if exc[0] is not None:
            wait_pipelines(self.handles)  # nothing may outlive its DMA
        return False


def wait_pipelines(handles: list) -> None:
    """Block until the deferred pipelined runs in `handles` have landed."""
    while handles:
        _prog, h, _keep = handles.pop(0)
        _C.pipeline_wait(h)


def run_segments_pipelined(prog, segments: List[List[torch.Tensor]],
                           out_specs: List[List[Tuple[tuple, torch.dtype]]]) -> List[List[torch.Tensor]]:
    """Pipelined H2D/compute/D2H over row chunks of several host segments.

    out_specs[s][j] = (full output shape, dtype) of fetch j for segment s.
    Inside `deferred_pipelines()` it returns before the outputs have landed.
    """
    dev = compute_device()
    segs = [[pin(t.contiguous()) for t in seg] for seg in segments]
    outs = [[empty_host(shape, dt, True) for (shape, dt) in spec] for spec in out_specs]
    total = sum(seg[0].shape[0] for seg in segs if seg)
    chunk = chunk_rows_for(segs[0], total) if segs and segs[0] else 1 << 16
    before = prog.stats()
    handles = getattr(_defer, "handles", None)
    with metrics.timer("pipelined"):
        h = prog.run_chunked(segs, outs, chunk, dev.index or 0, config.pipeline_depth, handles is None)
    if handles is not None:
        # the staged inputs and the outputs stay referenced until the wait
        handles.append((prog, h, (segs, outs)))
        metrics.add("pipelines_deferred")
    st = prog.stats()
    # this call's share of the program's cumulative counters; the *_device_ms
    # stage times come from hipEvent pairs around each chunk's copies/kernels
    metrics.add("chunks", st["chunks"] - before["chunks"])
    for k in ("h2d_ms", "compute_ms", "d2h_ms"):
        metrics.add("pipeline_" + k.replace("_ms", "_device_ms"), st[k] - before[k])
    return outs


def run_graph(graph_bytes: bytes, fetch_names: Sequence[str], feeds: Dict[str, object],
              device=None) -> List[np.ndarray]:
    """Evaluate fetches of a serialized graph on numpy/torch feeds (tf.Session.run)."""
    names = [str(n) for n in feeds]
    prog = program(graph_bytes, list(fetch_names), names)
    ins = []
    for n in names:
        v = feeds[n]
        ins.append(v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v, order="C")))
    dev = torch.device(device) if device is not None else compute_device()
    outs = run_program(prog, ins, dev)
    res = []
    for o in outs:
        a = o.cpu().numpy()
        res.append(a[()] if a.ndim == 0 else a)
    return res

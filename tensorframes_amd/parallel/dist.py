"""Process-group context: one process per GPU, partitions pinned to ranks.

The reference distributes work with Spark (mapPartitions tasks, Broadcast,
RDD.reduce to the driver, a groupBy shuffle; reference:
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:376-391,500,524,576).
Here every rank runs the same program (SPMD), owns partitions
``p % world_size == rank`` and exchanges data through the engine's own
communicators (parallel/comm.py): device tensors over RCCL / the one-shot
xGMI all-reduce, host tensors over a shared-memory segment when the ranks
share a node. torch.distributed is the bootstrap (rendezvous; gloo carries
the handful of host objects exchanged once) and the fallback
(`Config.collective_backend = "torch"`, ranks on several nodes).
"""
from __future__ import annotations

import datetime
import os
import pickle
import time
from typing import Any, List, Optional

import torch
import torch.distributed as dist

_state = {"device_group": None, "cpu_group": None, "initialized_here": False}


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def _forced() -> bool:
    from ..config import config
    return bool(config.force_collectives)


def is_distributed() -> bool:
    """True when cross-rank collectives run: a process group of world size > 1,
    or any group with `Config.force_collectives` (a 1-rank RCCL group on one
    GPU executes exactly the collective calls an 8-rank job makes)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or _forced()


def rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def world_size() -> int:
    return dist.get_world_size() if is_distributed() else 1


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", str(rank())))


def backend_name() -> Optional[str]:
    """The default process group's backend ("nccl" = RCCL, "gloo"), or None
    without a process group."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return str(dist.get_backend())


def init(backend: Optional[str] = None, timeout_s: Optional[float] = None, force: bool = False) -> bool:
    """Initialise the default process group from torchrun's env (idempotent).

    Collectives time out after `Config.collective_timeout_s`; RCCL errors and
    timeouts abort the communicator instead of hanging (async error handling).
    With `force` (or `Config.force_collectives`) a single process builds a
    world-size-1 group, so RCCL runs even on one GPU.
    Returns True when collectives are active (`is_distributed()`).
    """
    from ..config import config
    if timeout_s is None:
        timeout_s = config.collective_timeout_s
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if force:
        config.force_collectives = True
    if dist.is_initialized():
        _ensure_groups()
        return is_distributed()
    if env_world_size() <= 1 and not _forced():
        return False
    if env_world_size() <= 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
        if "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    use_gpu = torch.cuda.is_available()
    if backend is None:
        # TFA_DIST_BACKEND=gloo rehearses multi-rank logic where RCCL cannot
        # run (e.g. several ranks sharing one GPU)
        backend = os.environ.get("TFA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        torch.cuda.set_device(local_rank() % max(torch.cuda.device_count(), 1))
    kwargs = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl" and os.environ.get("TFA_NCCL_EAGER", "0") == "1":
        # eager RCCL communicator creation (errors surface at init); by default
        # the communicator is built at the first device collective, so jobs
        # that never issue one (the map_blocks benchmark) never create it
        kwargs["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(**kwargs)
    _state["initialized_here"] = True
    _ensure_groups()
    if is_distributed():
        from . import comm
        comm.init_host()  # collectively: every rank calls init
    return is_distributed()


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def gpu_local_cpus(device_index: Optional[int] = None) -> List[int]:
    """CPUs of the NUMA node closest to the GPU's PCIe root (sysfs
    ``local_cpulist``); [] when unknown."""
    import glob
    if not torch.cuda.is_available():
        return []
    idx = torch.cuda.current_device() if device_index is None else device_index
    p = torch.cuda.get_device_properties(idx)
    pattern = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.*"
    for d in sorted(glob.glob(pattern)):
        try:
            with open(os.path.join(d, "local_cpulist")) as f:
                return _parse_cpulist(f.read())
        except OSError:
            continue
    return []


def bind_numa(device_index: Optional[int] = None) -> List[int]:
    """Pin this process to the CPUs local to its GPU, so the page-locked
    staging buffers it allocates afterwards land on the GPU's NUMA node (one
    rank per GPU: each rank streams over its own PCIe link from local DRAM).
    Disabled with TFA_NUMA_BIND=0. Returns the CPU set applied ([] = none)."""
    if os.environ.get("TFA_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return []
    try:
        local = set(gpu_local_cpus(device_index))
        allowed = os.sched_getaffinity(0)
    except Exception:  # noqa: BLE001 - topology is best-effort
        return []
    cpus = sorted(local & allowed)
    if not cpus or set(cpus) == allowed:
        return []
    os.sched_setaffinity(0, cpus)
    if torch.get_num_threads() > len(cpus):
        torch.set_num_threads(len(cpus))
    return cpus


def _ensure_groups():
    if _state["device_group"] is None:
        _state["device_group"] = dist.group.WORLD
    if _state["cpu_group"] is None:
        if dist.get_backend() == "gloo":
            _state["cpu_group"] = dist.group.WORLD
        else:
            _state["cpu_group"] = dist.new_group(backend="gloo")


def shutdown():
    from . import comm
    comm.reset()
    if dist.is_initialized() and _state["initialized_here"]:
        dist.destroy_process_group()
    _state.update(device_group=None, cpu_group=None, initialized_here=False)


def owns(pid: int) -> bool:
    return pid % world_size() == rank()


def owner(pid: int) -> int:
    return pid % world_size()


def local_partitions(num_partitions: int) -> List[int]:
    r, w = rank(), world_size()
    return [p for p in range(num_partitions) if p % w == r]


def barrier():
    if is_distributed():
        shm = _host_comm()
        if shm is not None:
            with _traced("shm_barrier"):
                shm.barrier()
            return
        dist.barrier(group=_state["cpu_group"])


# -- bootstrap: torch.distributed's gloo group, never the engine communicators
#    (used while those are being built, and for the few objects exchanged once)
def all_reduce_bootstrap_(t: torch.Tensor, op: str = "Sum") -> torch.Tensor:
    if is_distributed():
        _ensure_groups()
        dist.all_reduce(t, op=_OPS[op], group=_state["cpu_group"])
    return t


def broadcast_bootstrap_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_distributed():
        _ensure_groups()
        dist.broadcast(t, src=src, group=_state["cpu_group"])
    return t


def barrier_bootstrap():
    if is_distributed():
        _ensure_groups()
        dist.barrier(group=_state["cpu_group"])


def _host_comm():
    """The shared-memory host communicator (built by init), or None."""
    from . import comm
    return comm.host()


_pending_events: List[tuple] = []  # (name, start, end) device events not yet read


class _traced:
    """Observability for one collective: a roctx range
    (`rocprofv3 --marker-trace` shows it next to the kernels) and metrics
    counters `collective_<name>` (calls), `collective_bytes`,
    `collective_ms` (host time: RCCL calls return once enqueued, gloo ones
    when done). Device collectives also record a hipEvent pair on the current
    stream; `collective_device_ms()` reads their elapsed device time (the
    RCCL kernel's own duration, not the enqueue time)."""

    def __init__(self, name: str, nbytes: int = 0, device: Optional[torch.device] = None):
        self.name, self.nbytes = name, int(nbytes)
        self.device = device if device is not None and device.type == "cuda" else None

    def __enter__(self):
        self.t0 = time.perf_counter()
        self.rng = torch.cuda.is_initialized()
        if self.rng:
            try:
                torch.cuda.nvtx.range_push(f"tfa.collective.{self.name}")
            except Exception:  # no roctx in this build
                self.rng = False
        self.ev = None
        if self.device is not None:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record(torch.cuda.current_stream(self.device))
        return self

    def __exit__(self, *exc):
        if self.ev is not None:
            self.ev[1].record(torch.cuda.current_stream(self.device))
            _pending_events.append((self.name,) + self.ev)
            if len(_pending_events) > 4096:
                collective_device_ms()
        if self.rng:
            torch.cuda.nvtx.range_pop()
        from ..utils.logging import metrics
        metrics.add(f"collective_{self.name}", 1)
        metrics.add("collective_bytes", self.nbytes)
        metrics.add("collective_ms", (time.perf_counter() - self.t0) * 1e3)
        return False


def collective_device_ms() -> float:
    """Device time of the device collectives issued so far (waits for them);
    also accumulated into metrics `collective_device_ms` and
    `collective_<name>_device_ms`."""
    from ..utils.logging import metrics
    total = 0.0
    while _pending_events:
        name, a, b = _pending_events.pop(0)
        b.synchronize()
        ms = a.elapsed_time(b)
        total += ms
        metrics.add("collective_device_ms", ms)
        metrics.add(f"collective_{name}_device_ms", ms)
    return metrics.snapshot().get("collective_device_ms", 0.0)


def _empty(shape, dtype, device) -> torch.Tensor:
    """Collective output buffers: the engine pool on a GPU (the collective
    runs on the current stream, which orders the pool block)."""
    from ..engine import device_empty
    return device_empty(shape, dtype, device)


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


# -- host-object collectives (small metadata / rows) over gloo
def all_gather_object(obj: Any) -> List[Any]:
    if not is_distributed():
        return [obj]
    _ensure_groups()
    out = [None] * world_size()
    with _traced("all_gather_object"):
        dist.all_gather_object(out, obj, group=_state["cpu_group"])
    return out


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_distributed():
        return obj
    _ensure_groups()
    box = [obj]
    with _traced("broadcast_object"):
        dist.broadcast_object_list(box, src=src, group=_state["cpu_group"])
    return box[0]


def all_to_all_objects(per_dest: List[Any]) -> List[Any]:
    """per_dest[r] goes to rank r; returns what each rank sent to us. A true
    pairwise exchange: the pickled payloads travel in one gloo all_to_all
    (each rank receives only its own share, not the whole shuffle)."""
    if not is_distributed():
        return [per_dest[0]]
    _ensure_groups()
    payload = [pickle.dumps(o, protocol=pickle.HIGHEST_PROTOCOL) for o in per_dest]
    sizes = all_to_all_counts([len(b) for b in payload])
    send = torch.frombuffer(bytearray(b"".join(payload)), dtype=torch.uint8) if any(payload) else \
        torch.empty(0, dtype=torch.uint8)
    shm = _host_comm()
    if shm is not None:
        with _traced("all_to_all_objects", _nbytes(send)):
            recv = shm.all_to_all_v(send, [len(b) for b in payload], sizes)
    else:
        recv = torch.empty(sum(sizes), dtype=torch.uint8)
        with _traced("all_to_all_objects", _nbytes(send)):
            dist.all_to_all_single(recv, send, sizes, [len(b) for b in payload], group=_state["cpu_group"])
    out, off, raw = [], 0, recv.numpy().tobytes()
    for n in sizes:
        out.append(pickle.loads(raw[off:off + n]))  # payloads written by our own ranks
        off += n
    return out


def gather_object(obj: Any, root: int = 0) -> Optional[List[Any]]:
    """Every rank's object on `root` (rank order); None elsewhere."""
    if not is_distributed():
        return [obj]
    _ensure_groups()
    out = [None] * world_size() if rank() == root else None
    with _traced("gather_object"):
        dist.gather_object(obj, out, dst=root, group=_state["cpu_group"])
    return out


def gather_rows(x: torch.Tensor, rows_per_rank: List[int], root: Optional[int] = None) -> Optional[List[torch.Tensor]]:
    """Variable-length row blocks of every rank (x: this rank's [rows, ...]
    host tensor, rows_per_rank known everywhere): each rank's block, in rank
    order, on every rank (root None) or only on `root` (None elsewhere).
    Balanced blocks go in one padded all_gather / gather of the tensor itself;
    skewed ones (padding would move > 25 % extra bytes) go rank by rank at
    their exact sizes (point-to-point to `root`, or one broadcast per rank).
    No pickling either way."""
    if not is_distributed():
        return [x]
    _ensure_groups()
    x = x.contiguous()
    rows = [int(r) for r in rows_per_rank]
    shm = _host_comm()
    if shm is not None:
        # every block at its exact size through the shared segment: to root
        # only (an all_to_all where only root receives), or to every rank
        w, me = world_size(), rank()
        with _traced("shm_gather_rows", _nbytes(x)):
            if root is None:
                got = shm.all_to_all_v(x.repeat((w,) + (1,) * (x.dim() - 1)) if w > 1 else x,
                                       [rows[me]] * w, rows)
            else:
                send = [rows[me] if r == root else 0 for r in range(w)]
                got = shm.all_to_all_v(x, send, rows if me == root else [0] * w)
        if root is not None and me != root:
            return None
        out, off = [], 0
        for r in rows:
            out.append(got[off:off + r])
            off += r
        return out
    mx = max(rows) if rows else 0
    if mx * len(rows) * 4 > sum(rows) * 5:
        return _gather_rows_exact(x, rows, root)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype)
    if x.shape[0]:
        pad[:x.shape[0]].copy_(x)
    group = _state["cpu_group"]
    with _traced("gather_rows", _nbytes(pad)):
        if root is None:
            parts = [torch.empty_like(pad) for _ in range(world_size())]
            dist.all_gather(parts, pad, group=group)
        else:
            parts = [torch.empty_like(pad) for _ in range(world_size())] if rank() == root else None
            dist.gather(pad, parts, dst=root, group=group)
    if parts is None:
        return None
    return [p[:int(r)] for p, r in zip(parts, rows_per_rank)]


def _gather_rows_exact(x: torch.Tensor, rows: List[int], root: Optional[int]) -> Optional[List[torch.Tensor]]:
    """gather_rows without padding: every block travels at its own size
    (zero-row ranks send nothing; every rank knows `rows`)."""
    group = _state["cpu_group"]
    me, tail = rank(), tuple(x.shape[1:])
    with _traced("gather_rows_exact", _nbytes(x)):
        if root is not None:
            if me != root:
                if rows[me]:
                    dist.send(x, dst=root, group=group)
                return None
            parts = []
            for r, n in enumerate(rows):
                if r == me:
                    parts.append(x)
                    continue
                buf = torch.empty((n,) + tail, dtype=x.dtype)
                if n:
                    dist.recv(buf, src=r, group=group)
                parts.append(buf)
            return parts
        parts = []
        for r, n in enumerate(rows):
            buf = x if r == me else torch.empty((n,) + tail, dtype=x.dtype)
            if n:
                dist.broadcast(buf, src=r, group=group)
            parts.append(buf)
        return parts


def broadcast_tensor(t: Optional[torch.Tensor], shape: tuple, dtype: torch.dtype, src: int) -> torch.Tensor:
    """`src`'s host tensor of a known shape/dtype on every rank (no pickling)."""
    if not is_distributed():
        return t
    _ensure_groups()
    buf = t.contiguous() if rank() == src else torch.empty(shape, dtype=dtype)
    shm = _host_comm()
    if shm is not None:
        with _traced("shm_broadcast", _nbytes(buf)):
            shm.broadcast(buf, src)
        return buf
    with _traced("broadcast", _nbytes(buf)):
        dist.broadcast(buf, src=src, group=_state["cpu_group"])
    return buf


# dtypes the shared-memory communicator folds (csrc/comm ShmComm fold_into);
# half / bfloat16 / bool reductions go to gloo
_SHM_REDUCE_DTYPES = {torch.float32, torch.float64, torch.int32, torch.int64, torch.int16, torch.uint8, torch.int8}


def all_reduce_host_(t: torch.Tensor, op: str = "Sum") -> torch.Tensor:
    """In-place all-reduce of a host tensor: the shared-memory communicator
    when the ranks share a node (and it folds the dtype), else the gloo group."""
    if not is_distributed():
        return t
    _ensure_groups()
    shm = _host_comm()
    if shm is not None and t.is_contiguous() and t.dtype in _SHM_REDUCE_DTYPES:
        with _traced("shm_all_reduce", _nbytes(t)):
            shm.all_reduce(t, op)
        return t
    dist.all_reduce(t, op=_OPS[op], group=_state["cpu_group"])
    return t


def all_to_all_counts(send_counts: List[int]) -> List[int]:
    """send_counts[r] = what we send to rank r; returns what each rank sends us."""
    if not is_distributed():
        return [int(send_counts[0])]
    _ensure_groups()
    t = torch.tensor([int(c) for c in send_counts], dtype=torch.int64)
    shm = _host_comm()
    if shm is not None:
        with _traced("shm_all_gather", _nbytes(t)):
            allc = shm.all_gather(t)  # [world, world]: row s = what rank s sends
        return allc[:, rank()].tolist()
    out = torch.empty_like(t)
    dist.all_to_all_single(out, t, group=_state["cpu_group"])
    return out.tolist()


def gpu_collectives() -> bool:
    """Device tensors can go straight to RCCL (False under a gloo rehearsal)."""
    _ensure_groups()
    return dist.get_backend(_state["device_group"]) == "nccl"


def all_to_all_tensors(chunks: List[torch.Tensor], recv_rows: List[int]) -> torch.Tensor:
    """chunks[r] (one dtype and trailing shape) goes to rank r; returns the
    received rows, concatenated in source-rank order. Device tensors move in
    ONE RCCL all_to_all over xGMI (the groupBy shuffle: SURVEY D4, reference
    DebugRowOps.scala:576), host tensors over gloo."""
    from ..engine import cat_rows
    x = cat_rows(chunks).contiguous()
    if not is_distributed():
        return x
    _ensure_groups()
    if x.is_cuda:
        ec = _engine_comm()
        if ec is not None and ec.rccl is not None:
            return ec.all_to_all_rows(x, [int(c.shape[0]) for c in chunks], recv_rows)
    if x.is_cuda and not gpu_collectives():
        return all_to_all_tensors([c.cpu() for c in chunks], recv_rows).to(x.device)
    if not x.is_cuda and _host_comm() is not None:
        with _traced("shm_all_to_all", _nbytes(x)):
            return _host_comm().all_to_all_v(x, [int(c.shape[0]) for c in chunks], [int(r) for r in recv_rows])
    group = _state["device_group"] if x.is_cuda else _state["cpu_group"]
    out = _empty((sum(recv_rows),) + tuple(x.shape[1:]), x.dtype, x.device)
    with _traced("all_to_all", _nbytes(x), x.device):
        dist.all_to_all_single(out, x, [int(r) for r in recv_rows], [int(c.shape[0]) for c in chunks],
                               group=group)
    return out


def all_to_all_rows(x: torch.Tensor, send_rows: List[int], recv_rows: List[int]) -> torch.Tensor:
    """Rows of x, already ordered by destination (send_rows[r] rows for rank
    r), exchanged in one all_to_all (no concatenation copy); returns the
    received rows in source-rank order."""
    if not is_distributed():
        return x
    _ensure_groups()
    x = x.contiguous()
    if x.is_cuda:
        ec = _engine_comm()
        if ec is not None and ec.rccl is not None:
            return ec.all_to_all_rows(x, send_rows, recv_rows)
    if x.is_cuda and not gpu_collectives():
        return all_to_all_rows(x.cpu(), send_rows, recv_rows).to(x.device)
    if not x.is_cuda and _host_comm() is not None:
        with _traced("shm_all_to_all", _nbytes(x)):
            return _host_comm().all_to_all_v(x, [int(r) for r in send_rows], [int(r) for r in recv_rows])
    group = _state["device_group"] if x.is_cuda else _state["cpu_group"]
    out = _empty((sum(recv_rows),) + tuple(x.shape[1:]), x.dtype, x.device)
    with _traced("all_to_all", _nbytes(x), x.device):
        dist.all_to_all_single(out, x, [int(r) for r in recv_rows], [int(c) for c in send_rows], group=group)
    return out


# -- tensor collectives: device tensors over RCCL, host tensors over gloo
_OPS = {"Sum": dist.ReduceOp.SUM, "Min": dist.ReduceOp.MIN, "Max": dist.ReduceOp.MAX,
        "Prod": dist.ReduceOp.PRODUCT}


def _engine_comm():
    from . import comm
    return comm.get()


def all_reduce_(t: torch.Tensor, op: str = "Sum") -> torch.Tensor:
    """In-place all-reduce. Device tensors go through the engine's own
    communicator (parallel/comm.py: one-shot IPC for <= 64 KB, its RCCL
    communicator above) when it serves them, else torch.distributed."""
    if not is_distributed():
        return t
    _ensure_groups()
    if t.is_cuda:
        ec = _engine_comm()
        if ec is not None and ec.can_all_reduce(t):
            return ec.all_reduce_(t.contiguous() if not t.is_contiguous() else t, op)
    if t.is_cuda and not gpu_collectives():  # gloo rehearsal: stage through the host
        return t.copy_(all_reduce_(t.cpu(), op))
    if not t.is_cuda and _host_comm() is not None and t.is_contiguous() and t.dtype in _SHM_REDUCE_DTYPES:
        with _traced("shm_all_reduce", _nbytes(t)):
            _host_comm().all_reduce(t, op)
        return t
    group = _state["device_group"] if t.is_cuda else _state["cpu_group"]
    with _traced("all_reduce", _nbytes(t), t.device):
        dist.all_reduce(t, op=_OPS[op], group=group)
    return t


def all_gather_tensor(t: torch.Tensor) -> torch.Tensor:
    """Stack the same-shaped tensor of every rank: [world, *t.shape]."""
    if not is_distributed():
        return t.unsqueeze(0)
    _ensure_groups()
    t = t.contiguous()
    if t.is_cuda:
        ec = _engine_comm()
        if ec is not None and ec.rccl is not None:
            return ec.all_gather(t)
    if t.is_cuda and not gpu_collectives():
        return all_gather_tensor(t.cpu()).to(t.device)
    if not t.is_cuda and _host_comm() is not None:
        with _traced("shm_all_gather", _nbytes(t)):
            return _host_comm().all_gather(t)
    if t.is_cuda:
        out = _empty((world_size(),) + tuple(t.shape), t.dtype, t.device)
        with _traced("all_gather", _nbytes(t), t.device):
            dist.all_gather_into_tensor(out, t, group=_state["device_group"])
        return out
    parts = [torch.empty_like(t) for _ in range(world_size())]
    with _traced("all_gather", _nbytes(t)):
        dist.all_gather(parts, t, group=_state["cpu_group"])
    return torch.stack(parts, 0)


# -- collective failure agreement
class RemoteRankError(RuntimeError):
    """Another rank failed in the local phase of a collective operator; this
    rank raises too instead of waiting in the next collective for
    `collective_timeout_s` (Spark fails the whole job on a task failure:
    reference DebugRowOps.scala:500, :524-525, :576)."""


class AgreedSoftFailure(RuntimeError):
    """Some rank hit a recoverable condition (a `soft` exception of `agreed`):
    every rank raises this so that all of them redo the operator together."""


def _raise_agreed(site: str, mine: Optional[BaseException], mine_status: int, statuses: List[tuple]):
    """statuses[r] = (status, kind, type name, message); 0 ok, 1 soft, 2 failed,
    3 only raised because another rank poisoned the communicator."""
    from ..utils.logging import metrics
    if any(st == 2 for st, *_ in statuses):
        metrics.add("collective_failures_agreed")
        if mine_status == 2:
            raise mine
        r, (_, kind, tname, text) = next((r, v) for r, v in enumerate(statuses) if v[0] == 2)
        if kind == "validation":
            from ..core import TensorFramesError
            raise TensorFramesError(f"{site} failed on rank {r}: {tname}: {text}")
        raise RemoteRankError(f"{site} failed on rank {r}: {tname}: {text}")
    metrics.add("collective_soft_failures")
    if mine_status == 1:
        raise mine
    raise AgreedSoftFailure(f"{site}: a rank asked for a collective retry")


def agreed(site: str, fn, soft: tuple = ()):
    """Runs `fn` -- the local phase of an SPMD operator, which may itself hold
    collectives; every rank calls this at the same point -- and agrees on the
    outcome, so that a rank that fails never leaves the others waiting in a
    collective for `collective_timeout_s`:

    * the common case costs ONE int64 Max all-reduce of a status word;
    * a rank whose `fn` raises poisons the shared-memory communicator at
      once, so every other rank's current or next host collective raises
      too; every rank then meets on the gloo bootstrap group, exchanges
      (status, error) and rank 0 clears the segment's barrier state;
    * a failure makes the failing rank re-raise its own error and every
      other rank raise RemoteRankError (TensorFramesError for a validation
      error) naming it; a `soft` exception on any rank (and no failure) makes
      every rank raise AgreedSoftFailure, so the caller redoes the operator
      together (the string-key collision fallback of aggregate).

    Without the shared-memory communicator (TFA_SHM_COLLECTIVES=0) the
    agreement is the status all-reduce alone, which covers failures that
    happen before `fn`'s first collective."""
    if not is_distributed():
        return fn()
    _ensure_groups()
    shm = _host_comm()
    res, err, status = None, None, 0
    try:
        res = fn()
    except BaseException as e:  # noqa: BLE001 - re-raised below on every rank
        err = e
        induced = shm is not None and shm.poisoned and isinstance(e, _C_collective_error())
        status = 3 if induced else (1 if soft and isinstance(e, soft) else 2)
        if shm is not None and status != 3:
            shm.poison()
    if shm is None:
        flag = torch.tensor([status], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=_state["cpu_group"])
        if int(flag.item()) == 0:
            return res
        text = "" if err is None else str(err)
        kind = "" if err is None else _classify(err)
        stats = [None] * world_size()
        dist.all_gather_object(stats, (status, kind, type(err).__name__ if err else "", text[:_MSG_BYTES]),
                               group=_state["cpu_group"])
        _raise_agreed(site, err, status, stats)
    if status == 0:
        try:
            flag = torch.tensor([0], dtype=torch.int64)
            shm.all_reduce(flag, "Max")
            if int(flag.item()) == 0:
                return res
        except _C_collective_error() as e:  # another rank failed and poisoned the segment
            err, status = e, 3
    # recovery on the bootstrap (gloo) group: every rank is out of the shm
    # communicator once it is here
    text = "" if err is None else str(err)
    kind = "" if err is None or status == 3 else _classify(err)
    stats = [None] * world_size()
    dist.all_gather_object(stats, (status, kind, type(err).__name__ if err else "", text[:_MSG_BYTES]),
                           group=_state["cpu_group"])
    dist.barrier(group=_state["cpu_group"])
    if rank() == 0:
        shm.reset_after_failure()
    dist.barrier(group=_state["cpu_group"])
    _raise_agreed(site, err, status, stats)


def _C_collective_error():
    from .comm import CollectiveError
    return CollectiveError


def _classify(e: BaseException) -> str:
    from ..utils import faults
    return faults.classify(e)


_MSG_BYTES = 1024

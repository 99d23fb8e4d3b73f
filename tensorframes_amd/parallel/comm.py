"""The engine's own communicators: collectives issued by the
native runtime, not through torch.distributed.

The reference has exactly two kinds of cross-partition traffic: the combine
of per-partition partials (`RDD.reduce` on the Spark driver, reference
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500, :524-525,
pairwise :732-750) and the groupBy shuffle (:576). Both run here on:

* `OneShotComm` (csrc/kernels/oneshot.hip) for device payloads <= 64 KB —
  every reduce_blocks / reduce_rows partial (one output cell, e.g. 4 KB): ONE
  hop, each GPU reading its peers' partials over its xGMI links in parallel,
  instead of a ring's 2(N-1) dependent hops. Its buffers are allocated
  uncached, peer access is checked for every pair of GPUs, and a start-up
  self-test (rank-tagged all-reduces, checked on every rank, agreed on by all)
  decides whether it is used at all; otherwise every rank uses RCCL.
* `RcclComm` — an RCCL communicator of the engine's own (ncclCommInitRank;
  the 128-byte unique id rides on the bootstrap process group) for large
  all-reduces, all-gathers and the grouped send/recv all-to-all shuffle.
  Only built when every rank has a GPU of its own (RCCL rejects two ranks on
  one device).
* `ShmComm` — host tensors of the ranks of one node through a shared-memory
  segment: the whole data path of CPU-only multi-process jobs and the
  row-count / flag exchanges of GPU jobs (gloo's TCP loopback is only the
  bootstrap).
* `FakeComm` — N in-process ranks (threads): the C++ contract test double.

Failure detection (the reference's counterpart is Spark's task
failure around RDD.reduce and the shuffle): every collective is bounded by
`Config.collective_timeout_s`. A rank that waits past it raises
`CollectiveError`; an RCCL collective nobody waits on is caught by the
communicator's watchdog thread, which aborts the communicator and ends the
process with status `EXIT_COLLECTIVE_TIMEOUT` (`Config.collective_timeout_exit`)
so the launcher tears the job down.

torch.distributed stays the bootstrap (rendezvous, store, the ids and IPC
handles exchanged once). `Config.collective_backend = "torch"` routes every
collective back through torch.distributed (A/B and fallback).
"""
from __future__ import annotations

import os
import socket
import threading
import uuid
from typing import List, Optional

import torch

from .._native import _C
from ..utils.logging import logger, metrics
from . import dist

CollectiveError = _C.CollectiveError
EXIT_COLLECTIVE_TIMEOUT = int(_C.EXIT_COLLECTIVE_TIMEOUT)

_lock = threading.Lock()
_state = {"key": None, "comm": None, "host_key": None, "host": None}
_ONESHOT_DTYPES = (torch.float32, torch.float64, torch.int32, torch.int64)


class EngineComm:
    """Per-process device communicator: one-shot small all-reduce + RCCL."""

    def __init__(self, rank: int, size: int, device: int, oneshot=None, rccl=None):
        self.rank, self.size, self.device = rank, size, device
        self.oneshot = oneshot
        self.rccl = rccl

    @property
    def kinds(self) -> List[str]:
        return [k for k, v in (("oneshot", self.oneshot), ("rccl", self.rccl)) if v is not None]

    def _small(self, t: torch.Tensor) -> bool:
        return (self.oneshot is not None and t.dtype in _ONESHOT_DTYPES
                and t.numel() * t.element_size() <= _C.OneShotComm.max_bytes())

    def can_all_reduce(self, t: torch.Tensor) -> bool:
        if not t.is_cuda or t.device.index != self.device:
            return False
        return self._small(t) or self.rccl is not None

    def all_reduce_(self, t: torch.Tensor, op: str = "Sum") -> torch.Tensor:
        """In place on the current stream: one-shot for <= 64 KB, else RCCL."""
        from .dist import _traced
        if self._small(t):
            with _traced("oneshot_all_reduce", t.numel() * t.element_size(), t.device):
                self.oneshot.all_reduce(t, op)
            return t
        with _traced("rccl_all_reduce", t.numel() * t.element_size(), t.device):
            self.rccl.all_reduce(t, op)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        from .dist import _traced
        with _traced("rccl_all_gather", t.numel() * t.element_size(), t.device):
            return self.rccl.all_gather(t.contiguous())

    def all_to_all_rows(self, x: torch.Tensor, send_rows: List[int], recv_rows: List[int]) -> torch.Tensor:
        from .dist import _traced
        with _traced("rccl_all_to_all", x.numel() * x.element_size(), x.device):
            return self.rccl.all_to_all_v(x.contiguous(), [int(r) for r in send_rows], [int(r) for r in recv_rows])

    def wait(self) -> None:
        """Bounded wait for the RCCL collectives issued so far (raises
        CollectiveError past `collective_timeout_s`)."""
        if self.rccl is not None:
            self.rccl.wait()

    def check(self) -> None:
        """Raises CollectiveError if a one-shot flag wait timed out or the RCCL
        communicator failed (call after the stream has been synchronised)."""
        if self.oneshot is not None and self.oneshot.calls:
            self.oneshot.check()
        if self.rccl is not None:
            self.rccl.check()


def _device_identity(idx: int) -> str:
    p = torch.cuda.get_device_properties(idx)
    uuid_ = getattr(p, "uuid", None)
    return str(uuid_) if uuid_ is not None else f"{p.pci_domain_id}:{p.pci_bus_id}:{p.pci_device_id}"


def _visible_index(ident: str) -> Optional[int]:
    """This process's index of the device with identity `ident` (None if not visible)."""
    for i in range(torch.cuda.device_count()):
        if _device_identity(i) == ident:
            return i
    return None


def _agree(ok: bool) -> bool:
    """Every rank's verdict over the bootstrap group: True only if all say True."""
    flag = torch.tensor([int(ok)], dtype=torch.int64)
    dist.all_reduce_bootstrap_(flag, "Min")
    return bool(int(flag.item()))


def _oneshot_self_test(os_comm, rank: int, size: int, dev: int) -> Optional[str]:
    """Rank-tagged all-reduces through the one-shot path, checked on this
    rank: both buffer slots, two dtypes, every element. None when correct,
    else the reason. TFA_ONESHOT_SELFTEST_FAIL=1 forces a failure (tests)."""
    from ..config import config
    try:
        os_comm.set_timeout(min(10.0, float(config.collective_timeout_s)))
        n = 1027
        idx = torch.arange(n, dtype=torch.int64, device=f"cuda:{dev}")
        want_i = (idx + 1) * (size * (size + 1) // 2)
        for e in range(3):  # slots 1, 0, 1
            t = (idx + 1) * (rank + 1)
            os_comm.all_reduce(t, "Sum")
            tf = torch.full((257,), float(rank + 1) * (e + 1), dtype=torch.float64, device=f"cuda:{dev}")
            os_comm.all_reduce(tf, "Max")
            torch.cuda.synchronize(dev)
            os_comm.check()
            if not torch.equal(t, want_i):
                return f"Sum mismatch on pass {e}"
            if not bool((tf == float(size) * (e + 1)).all()):
                return f"Max mismatch on pass {e}"
        if os.environ.get("TFA_ONESHOT_SELFTEST_FAIL", "0") == "1":
            return "forced by TFA_ONESHOT_SELFTEST_FAIL"
        return None
    except Exception as ex:  # noqa: BLE001 - any failure disables the path
        return f"{type(ex).__name__}: {ex}"
    finally:
        try:
            os_comm.set_timeout(float(config.collective_timeout_s))
        except Exception:  # noqa: BLE001
            pass


def get() -> Optional[EngineComm]:
    """The process's device communicator (built on first use, collectively:
    every rank must reach the first device collective together, which the SPMD
    operators guarantee). None when collectives are off, there is no GPU, or
    `Config.collective_backend` is "torch"."""
    from ..config import config
    from .. import engine
    if config.collective_backend == "torch" or not dist.is_distributed() or not engine.gpu_available():
        return None
    key = (id(torch.distributed.group.WORLD), dist.world_size(), dist.rank())
    with _lock:
        if _state["key"] == key:
            return _state["comm"]
    dev = engine.compute_device().index or 0
    rank, size = dist.rank(), dist.world_size()
    # which ranks share a device (RCCL needs one device per rank) and whether
    # every pair of distinct GPUs can reach each other (one-shot path)
    ids = dist.all_gather_object(_device_identity(dev))
    own_devices = len(set(ids)) == len(ids)
    oneshot = None
    if size <= 8 and config.oneshot_allreduce:
        peer_ok = True
        for ident in set(ids):
            j = _visible_index(ident)
            if j is not None and j != dev and not _C.can_access_peer(dev, j):
                peer_ok = False
        mine = None
        reason = None if peer_ok else "no peer access between two of the ranks' GPUs"
        if peer_ok:
            mine = _C.OneShotComm(rank, size, dev)
            handles = dist.all_gather_object(mine.ipc_handle())
            try:
                mine.open(list(handles))
            except Exception as ex:  # noqa: BLE001 - IPC unavailable: RCCL only
                reason = f"IPC open failed: {ex}"
        # every rank must agree to use it (one failing open disables it everywhere)
        if _agree(reason is None):
            reason = _oneshot_self_test(mine, rank, size, dev)
            if _agree(reason is None):
                oneshot = mine
                mine.set_timeout(float(config.collective_timeout_s))
                metrics.add("oneshot_selftest_ok")
            else:
                reason = reason or "another rank's self-test failed"
        else:
            reason = reason or "another rank could not open the peer buffers"
        if oneshot is None:
            metrics.add("oneshot_selftest_failed")
            logger.warning("one-shot all-reduce disabled (%s); small all-reduces use RCCL", reason)
        else:
            logger.info("one-shot all-reduce enabled (%s buffers)", mine.alloc_kind)
    rccl = None
    if own_devices and dist.backend_name() == "nccl":
        uid = dist.broadcast_object(_C.rccl_unique_id() if rank == 0 else None, src=0)
        rccl = _C.RcclComm(uid, rank, size, dev)
        rccl.set_timeout(float(config.collective_timeout_s), bool(config.collective_timeout_exit))
    c = EngineComm(rank, size, dev, oneshot, rccl) if (oneshot or rccl) else None
    with _lock:
        _state.update(key=key, comm=c)
    return c


def _node_identity() -> str:
    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    return f"{socket.gethostname()}/{boot}"


def init_host() -> Optional["_C.ShmComm"]:
    """Build the shared-memory host communicator (collectively, from
    dist.init): rank 0 creates the segment, the others attach, then it is
    unlinked (the mappings stay valid; a crashed job leaves nothing behind in
    /dev/shm). Returns None when the ranks are not on one node, the feature is
    off, or any rank fails to map the segment."""
    from ..config import config
    if config.collective_backend == "torch" or not config.shm_collectives or not dist.is_distributed():
        return None
    key = (id(torch.distributed.group.WORLD), dist.world_size(), dist.rank())
    with _lock:
        if _state["host_key"] == key:
            return _state["host"]
    rank, size = dist.rank(), dist.world_size()
    nodes = dist.all_gather_object(_node_identity())
    shm = None
    if len(set(nodes)) == 1 and size <= 64:
        name = dist.broadcast_object(f"/tfa_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None, src=0)
        slot = int(config.shm_slot_bytes)
        err = None
        if rank == 0:
            try:
                shm = _C.ShmComm(name, 0, size, slot, True)
            except Exception as ex:  # noqa: BLE001
                err = ex
        created = torch.tensor([int(shm is not None)], dtype=torch.int64)
        dist.broadcast_bootstrap_(created, 0)  # the others attach only to a segment that exists
        if int(created.item()) and rank != 0:
            try:
                shm = _C.ShmComm(name, rank, size, slot, False)
            except Exception as ex:  # noqa: BLE001
                err = ex
        ok = _agree(shm is not None)
        if shm is not None and rank == 0:
            shm.unlink()  # every rank has mapped it (or gave up): nothing stays in /dev/shm
        if not ok:
            logger.warning("shared-memory collectives disabled%s", f": {err}" if err is not None else "")
            shm = None
        else:
            shm.set_timeout(float(config.collective_timeout_s))
    with _lock:
        _state.update(host_key=key, host=shm)
    return shm


def check_built() -> None:
    """Raise CollectiveError if the already-built device communicator has a
    failed collective (one-shot flag timeout, RCCL timeout / async error).
    Never builds one. Call after synchronising on a collective's result."""
    with _lock:
        c = _state["comm"]
    if c is not None:
        c.check()


def host() -> Optional["_C.ShmComm"]:
    """The shared-memory host communicator if dist.init built one (never
    builds it: host collectives may run before or without it)."""
    key = (id(torch.distributed.group.WORLD), dist.world_size(), dist.rank()) if dist.is_distributed() else None
    with _lock:
        return _state["host"] if key is not None and _state["host_key"] == key else None


def reset() -> None:
    with _lock:
        _state.update(key=None, comm=None, host_key=None, host=None)

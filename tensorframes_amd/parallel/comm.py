"""The engine's own communicator: device collectives issued by
the native runtime on the engine's stream, not through torch.distributed.

The reference has exactly two kinds of cross-partition traffic: the combine
of per-partition partials (`RDD.reduce` on the Spark driver, reference
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500, :524-525,
pairwise :732-750) and the groupBy shuffle (:576). Both run here on:

* `OneShotComm` (csrc/kernels/oneshot.hip) for payloads <= 64 KB — every
  reduce_blocks / reduce_rows partial (one output cell, e.g. 4 KB): ONE hop,
  each GPU reading its peers' partials over its xGMI links in parallel,
  instead of a ring's 2(N-1) dependent hops. It also works for ranks that
  share a GPU (the 2-ranks-on-one-GPU rehearsal).
* `RcclComm` — an RCCL communicator of the engine's own (ncclCommInitRank;
  the 128-byte unique id rides on the bootstrap process group) for large
  all-reduces, all-gathers and the grouped send/recv all-to-all shuffle.
  Only built when every rank has a GPU of its own (RCCL rejects two ranks on
  one device).
* `FakeComm` — N in-process ranks (threads): the CPU test double
  (tests/test_comm.py runs the collective contract at N = 2/4/8).

torch.distributed stays the bootstrap (rendezvous, store) and the host-object
channel (gloo), the role Spark's driver RPC plays in the reference.
`Config.collective_backend = "torch"` routes device collectives back through
torch.distributed (A/B and fallback).
"""
from __future__ import annotations

import threading
from typing import List, Optional

import torch

from .._native import _C
from . import dist

_lock = threading.Lock()
_state = {"key": None, "comm": None}


class EngineComm:
    """Per-process device communicator: one-shot small all-reduce + RCCL."""

    def __init__(self, rank: int, size: int, device: int, oneshot=None, rccl=None):
        self.rank, self.size, self.device = rank, size, device
        self.oneshot = oneshot
        self.rccl = rccl

    @property
    def kinds(self) -> List[str]:
        return [k for k, v in (("oneshot", self.oneshot), ("rccl", self.rccl)) if v is not None]

    def can_all_reduce(self, t: torch.Tensor) -> bool:
        if not t.is_cuda or t.device.index != self.device:
            return False
        small = self.oneshot is not None and t.numel() * t.element_size() <= _C.OneShotComm.max_bytes() \
            and t.dtype in (torch.float32, torch.float64, torch.int32, torch.int64)
        return small or self.rccl is not None

    def all_reduce_(self, t: torch.Tensor, op: str = "Sum") -> torch.Tensor:
        """In place on the current stream: one-shot for <= 64 KB, else RCCL."""
        from .dist import _traced
        if self.oneshot is not None and t.numel() * t.element_size() <= _C.OneShotComm.max_bytes() \
                and t.dtype in (torch.float32, torch.float64, torch.int32, torch.int64):
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

    def check(self) -> None:
        """Raises if a one-shot flag wait timed out (call after the stream sync)."""
        if self.oneshot is not None and self.oneshot.calls:
            self.oneshot.check()


def _device_identity(idx: int) -> str:
    p = torch.cuda.get_device_properties(idx)
    uuid = getattr(p, "uuid", None)
    return str(uuid) if uuid is not None else f"{p.pci_domain_id}:{p.pci_bus_id}:{p.pci_device_id}"


def get() -> Optional[EngineComm]:
    """The process's engine communicator (built on first use, collectively:
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
    # the node is small enough for the one-shot path
    ids = dist.all_gather_object(_device_identity(dev))
    own_devices = len(set(ids)) == len(ids)
    oneshot = None
    if size <= 8 and config.oneshot_allreduce:
        mine = _C.OneShotComm(rank, size, dev)
        handles = dist.all_gather_object(mine.ipc_handle())
        ok = True
        try:
            mine.open(list(handles))
        except Exception:  # noqa: BLE001 - IPC unavailable: RCCL only
            ok = False
        # every rank must agree to use it (one failing open disables it everywhere)
        flag = torch.tensor([int(ok)], dtype=torch.int64)
        dist.all_reduce_host_(flag, "Min")
        oneshot = mine if int(flag.item()) else None
    rccl = None
    if own_devices and dist.backend_name() == "nccl":
        uid = dist.broadcast_object(_C.rccl_unique_id() if rank == 0 else None, src=0)
        rccl = _C.RcclComm(uid, rank, size, dev)
    c = EngineComm(rank, size, dev, oneshot, rccl) if (oneshot or rccl) else None
    with _lock:
        _state.update(key=key, comm=c)
    return c


def reset() -> None:
    with _lock:
        _state.update(key=None, comm=None)

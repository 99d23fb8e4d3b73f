"""Failure handling for partition tasks: bounded retries and fault injection.

The reference relied on Spark task retry / lineage re-execution and had no
fault hooks of its own. Here a partition task is a
deterministic function of its input block, so a task that fails with a
runtime (non-validation) error can be re-run; `Config.task_retries` bounds the
attempts (0 = fail fast, the default). `inject` arms a fault at a named site
for tests, e.g. "the map_blocks task of partition 3 fails once":

    with faults.inject("map_blocks", partition=3, times=1):
        df2.collect()          # retried when config.task_retries >= 1

Validation errors (TensorFramesError and other ValueError/TypeError that do
not come from the device runtime) are never retried.
"""
from __future__ import annotations

import contextlib
import threading
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Optional

from .logging import logger, metrics


class InjectedFault(RuntimeError):
    """Raised by an armed injection site."""


@dataclass
class _Fault:
    site: str
    partition: Optional[int]
    rank: Optional[int]
    times: int
    exc: type


_lock = threading.Lock()
_armed: List[_Fault] = []


@contextlib.contextmanager
def inject(site: str, partition: Optional[int] = None, times: int = 1, rank: Optional[int] = None,
           exc: type = InjectedFault):
    """Arm a fault at `site` ("map_blocks", "map_rows", "reduce_blocks",
    "reduce_rows", "aggregate") for `partition` (None = any) on `rank`
    (None = any), firing `times` times."""
    f = _Fault(site, partition, rank, times, exc)
    with _lock:
        _armed.append(f)
    try:
        yield f
    finally:
        with _lock:
            if f in _armed:
                _armed.remove(f)


def check(site: str, partitions: Iterable[int]):
    """Injection point: raise if a fault is armed for `site` and one of `partitions`."""
    if not _armed:
        return
    from ..parallel import dist
    r = dist.rank()
    with _lock:
        for f in _armed:
            if f.site != site or f.times <= 0 or (f.rank is not None and f.rank != r):
                continue
            hit = [p for p in partitions if f.partition is None or p == f.partition]
            if hit:
                f.times -= 1
                metrics.add("faults_injected")
                raise f.exc(f"injected fault at {site} (partition {hit[0]}, rank {r})")


def is_retryable(e: BaseException) -> bool:
    from ..core import TensorFramesError
    if isinstance(e, (TensorFramesError, TypeError, KeyError)):
        return False
    if isinstance(e, ValueError):
        # native runtime errors surface as GraphError (a ValueError); only the
        # device-side ones (HIP launch/runtime failures) are transient
        msg = str(e).lower()
        return "hip" in msg or "device" in msg
    return isinstance(e, (RuntimeError, OSError, MemoryError))


def with_retries(site: str, fn: Callable[[Dict[int, object]], Dict[int, object]]):
    """Wraps a partition-task function {pid: block} -> {pid: block}: on a
    retryable failure each partition is re-run alone, up to
    `config.task_retries` times."""
    from ..config import config

    def run(blocks):
        try:
            check(site, blocks.keys())
            return fn(blocks)
        except Exception as e:  # noqa: BLE001
            if config.task_retries <= 0 or not is_retryable(e):
                raise
            first = e
        logger.warning("%s: task failed (%s); retrying %d partition(s) one by one", site, first, len(blocks))
        res = {}
        for pid in sorted(blocks):
            for attempt in range(1, config.task_retries + 1):
                try:
                    check(site, [pid])
                    res.update(fn({pid: blocks[pid]}))
                    metrics.add("task_retries")
                    break
                except Exception as e:  # noqa: BLE001
                    if attempt >= config.task_retries or not is_retryable(e):
                        raise
                    logger.warning("%s: partition %d attempt %d failed: %s", site, pid, attempt, e)
        return res

    return run

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
not come from the device runtime) are never retried. Device errors are
sorted: running out of memory is recoverable (cached blocks are released and
the partition re-run); a HIP fault (illegal address, kernel abort, ECC...)
leaves the process's GPU context unusable, so it is NEVER retried in-process:
it is re-raised at once as `DeviceFaultError`, naming the node and kernel the
executor was running (csrc/runtime/executor.cpp checks every launch). Other
HIP errors (an invalid launch configuration, ...) are deterministic and not
retried either.

Recovery from a sticky fault happens one level up, in a fresh process: a rank
whose entry point is wrapped in `exit_on_device_fault` exits with
`EXIT_DEVICE_FAULT`, and the launcher (`parallel/launch.py`, `max_restarts` /
`TFA_MAX_RESTARTS`) re-runs the whole job in new processes with new HIP
contexts. Partition tasks are deterministic functions of their input
partitions, so the re-run recomputes the same results (the reference's
counterpart is Spark's task re-execution from lineage).
"""
from __future__ import annotations

import contextlib
import threading
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Optional

from .logging import logger, metrics


class InjectedFault(RuntimeError):
    """Raised by an armed injection site."""


class DeviceFaultError(RuntimeError):
    """A sticky GPU fault: the HIP context of this process is lost. The job
    must fail (or be re-run in a fresh process); retrying here would fail
    again or hang."""


# substrings of HIP/HSA errors after which the context cannot be used again
_STICKY = ("illegal address", "illegaladdress", "memory access fault", "launch failure", "launchfailure",
           "device-side assert", "hiperrorassert", "illegal instruction", "illegalinstruction", "ecc",
           "hardware exception", "hsa_status_error", "launch timed out", "launchtimeout", "misaligned address",
           "context is destroyed", "contextisdestroyed", "unspecified launch")
_OOM = ("out of memory", "outofmemory", "hiperroroutofmemory", "memoryallocation")


def classify(e: BaseException) -> str:
    """'validation', 'oom', 'sticky', 'device' (other deterministic HIP errors),
    'transient' (injected faults, I/O, other runtime errors)."""
    from ..core import TensorFramesError
    if isinstance(e, DeviceFaultError):
        return "sticky"
    if isinstance(e, MemoryError):
        return "oom"
    msg = str(e).lower()
    if any(k in msg for k in _STICKY):
        return "sticky"
    if any(k in msg for k in _OOM):
        return "oom"
    if isinstance(e, (TensorFramesError, TypeError, KeyError)):
        return "validation"
    if "hip error" in msg or "hiperror" in msg:
        return "device"
    if isinstance(e, ValueError):
        return "validation"
    if isinstance(e, InjectedFault):
        return "transient"
    return "transient" if isinstance(e, (RuntimeError, OSError)) else "validation"


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


EXIT_DEVICE_FAULT = 75  # exit status of a rank that lost its GPU context


def exit_on_device_fault(fn: Callable):
    """Decorator for a rank's entry point: a sticky GPU fault ends the process
    with `EXIT_DEVICE_FAULT` (after logging it), so a supervising launcher can
    re-run the job in fresh processes; other errors propagate unchanged."""
    import functools

    @functools.wraps(fn)
    def run(*a, **kw):
        try:
            return fn(*a, **kw)
        except Exception as e:  # noqa: BLE001
            if classify(e) != "sticky":
                raise
            logger.error("device fault, exiting for a fresh-process restart: %s", e)
            import sys
            sys.stderr.flush()
            raise SystemExit(EXIT_DEVICE_FAULT) from e
    return run


def restart_count() -> int:
    """How many times the launcher has re-run this job (0 = first attempt)."""
    import os
    return int(os.environ.get("TFA_RESTART_COUNT", "0"))


def is_retryable(e: BaseException) -> bool:
    return classify(e) in ("oom", "transient")


def _raise_sticky(site: str, e: BaseException):
    metrics.add("device_faults")
    if isinstance(e, DeviceFaultError):
        raise e
    raise DeviceFaultError(f"{site}: GPU fault, the device context of this process is lost and the task is "
                           f"not retried in-process: {e}") from e


def _release_device_memory():
    try:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.empty_cache()
    except Exception:  # noqa: BLE001 - best effort before a retry
        pass


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
            if classify(e) == "sticky":
                _raise_sticky(site, e)
            if config.task_retries <= 0 or not is_retryable(e):
                raise
            if classify(e) == "oom":
                _release_device_memory()
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
                    if classify(e) == "sticky":
                        _raise_sticky(site, e)
                    if attempt >= config.task_retries or not is_retryable(e):
                        raise
                    if classify(e) == "oom":
                        _release_device_memory()
                    logger.warning("%s: partition %d attempt %d failed: %s", site, pid, attempt, e)
        return res

    return run

"""Single-node multi-process launcher: one process per GPU.

`python bench.py --gpus 8` (or any script that calls `spawn_if_needed`) must
not run one process on one GPU: the parent process re-runs the same script as
N fresh child processes, one rank each, with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set (the torchrun contract), and waits for them.

The parent never touches the GPU (no HIP call, no `torch.cuda.is_available()`),
and children are started as new processes (`subprocess`, never `exec*`), so a
launcher parent is safe on hosts where replacing a GPU-initialised process is
forbidden. When the script already runs under torchrun (WORLD_SIZE set) the
launcher does nothing.

Reference counterpart: every TensorFrames operator is a Spark job whose tasks
run on all executors (reference: src/main/scala/org/tensorframes/impl/DebugRowOps.scala:376-392);
here the executors are ranks pinned 1:1 to GPUs.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def under_launcher() -> bool:
    """True when this process is one rank of a multi-process job."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


EXIT_DEVICE_FAULT = 75  # == utils.faults.EXIT_DEVICE_FAULT (not imported: no package import here)


def spawn(argv: Sequence[str], nprocs: int, extra_env: Optional[Dict[str, str]] = None,
          timeout_s: Optional[float] = None, max_restarts: Optional[int] = None) -> int:
    """Run `python argv...` as `nprocs` ranks on this node; returns the first
    non-zero exit code (0 when every rank succeeded). A failing rank takes
    the others down (they would block in a collective otherwise).

    When a rank exits with EXIT_DEVICE_FAULT (it lost its GPU context, see
    `faults.exit_on_device_fault`) the whole job is re-run in fresh processes,
    up to `max_restarts` times (default: TFA_MAX_RESTARTS, else 0); each
    attempt sees TFA_RESTART_COUNT."""
    if max_restarts is None:
        max_restarts = int(os.environ.get("TFA_MAX_RESTARTS", "0"))
    attempt = 0
    while True:
        env = dict(extra_env or {})
        env["TFA_RESTART_COUNT"] = str(attempt)
        rc = _spawn_once(argv, nprocs, env, timeout_s)
        if rc != EXIT_DEVICE_FAULT or attempt >= max_restarts:
            return rc
        attempt += 1
        print(f"[launch] a rank lost its GPU context (exit {rc}); restarting the job "
              f"({attempt}/{max_restarts})", file=sys.stderr, flush=True)


def _spawn_once(argv: Sequence[str], nprocs: int, extra_env: Dict[str, str], timeout_s: Optional[float]) -> int:
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env, start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    _terminate(live)
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                _terminate(live)
                return rc or 124
            time.sleep(0.05)
    except KeyboardInterrupt:
        _terminate(live)
        raise
    return rc


def _terminate(procs: List[subprocess.Popen], grace_s: float = 10.0) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)  # each child leads its own session
            except OSError:
                pass
    deadline = time.monotonic() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass


def spawn_if_needed(nprocs: int, argv: Optional[Sequence[str]] = None,
                    extra_env: Optional[Dict[str, str]] = None) -> Optional[int]:
    """If `nprocs` > 1 and this process is not already a rank, run the current
    script as `nprocs` ranks and return the job's exit code; otherwise return
    None (the caller is a rank, or a single-process run, and goes on)."""
    if nprocs <= 1 or under_launcher():
        return None
    return spawn(list(argv) if argv is not None else [sys.argv[0]] + sys.argv[1:], nprocs, extra_env)

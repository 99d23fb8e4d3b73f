"""Latency of the device all-reduce paths: the engine's one-shot
IPC all-reduce, the engine's own RCCL communicator, and torch.distributed's
RCCL, for payloads from one element to 16 MB (a reduce_blocks partial is one
output cell: 4 KB for f32[1024]).

    python scripts/comm_bench.py                      # world size 1 (one GPU)
    TFA_DIST_BACKEND=gloo torchrun --nproc-per-node 2 scripts/comm_bench.py
        # 2 ranks sharing one GPU: one-shot only (RCCL refuses a shared device)

Prints one JSON line per (path, bytes): median microseconds per call, host
wall time of `iters` back-to-back calls closed by a stream synchronisation.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorframes_amd.config import config  # noqa: E402
from tensorframes_amd.parallel import comm, dist  # noqa: E402


def bench(fn, t, iters=200, reps=5):
    for _ in range(20):
        fn(t)
    torch.cuda.synchronize()
    best = []
    for _ in range(reps):
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn(t)
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t0) / iters * 1e6)
    best.sort()
    return best[len(best) // 2]


def main():
    dist.init(force=True)
    dev = torch.device("cuda", dist.local_rank() % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ec = comm.get()
    rank, world = dist.rank(), dist.world_size()
    sizes = [4, 4096, 65536, 1 << 20, 16 << 20]
    for nb in sizes:
        t = torch.ones(nb // 4, dtype=torch.float32, device=dev)
        paths = []
        if ec is not None and ec.oneshot is not None and nb <= ec.oneshot.max_bytes():
            paths.append(("engine_oneshot", lambda x: ec.oneshot.all_reduce(x, "Sum")))
        if ec is not None and ec.rccl is not None:
            paths.append(("engine_rccl", lambda x: ec.rccl.all_reduce(x, "Sum")))
        if dist.gpu_collectives():
            import torch.distributed as tdist
            paths.append(("torch_rccl", lambda x: tdist.all_reduce(x)))
        for name, fn in paths:
            us = bench(fn, t)
            if rank == 0:
                print(json.dumps({"path": name, "bytes": nb, "world": world, "us_per_call": round(us, 2),
                                  "backend": dist.backend_name(), "oneshot": config.oneshot_allreduce}),
                      flush=True)
    if ec is not None:
        ec.check()
    dist.shutdown()


if __name__ == "__main__":
    main()

"""Bidirectional pinned-DMA throughput with 1 or 2 copy streams per direction
(is the headline's H2D+D2H pipeline bound by the link or by one DMA queue?).

    python scripts/pcie_streams_probe.py
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    nbytes = 256 << 20
    reps = 8
    res = {}
    for per_dir in (1, 2, 3):
        hs = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(per_dir)]
        ho = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(per_dir)]
        ds = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(per_dir)]
        do = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(per_dir)]
        up = [torch.cuda.Stream(dev) for _ in range(per_dir)]
        down = [torch.cuda.Stream(dev) for _ in range(per_dir)]
        for mode in ("h2d", "d2h", "bidir"):
            for it in range(2):  # warm, timed
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    for i in range(per_dir):
                        if mode in ("h2d", "bidir"):
                            with torch.cuda.stream(up[i]):
                                ds[i].copy_(hs[i], non_blocking=True)
                        if mode in ("d2h", "bidir"):
                            with torch.cuda.stream(down[i]):
                                ho[i].copy_(do[i], non_blocking=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            moved = reps * per_dir * nbytes * (2 if mode == "bidir" else 1)
            res[f"{mode}_{per_dir}streams_GBps"] = moved / dt / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()

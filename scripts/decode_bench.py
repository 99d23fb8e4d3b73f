"""Host JPEG decode throughput of the map_rows image path
(ops/host_ops.decode_image on a thread pool), on the synthetic images of
examples/read_image.py. Prints one line per thread count.

    python scripts/decode_bench.py [--images N] [--threads 1,4,8,16]
"""
import argparse
import io
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tensorframes_amd.ops.host_ops import decode_image  # noqa: E402


def main():
    from PIL import Image
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=1024)
    ap.add_argument("--threads", default="1,2,4,8,12,16")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    jp = []
    for _ in range(a.images):
        h, w = rng.integers(180, 400, 2)
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(buf, format="JPEG", quality=90)
        jp.append(bytearray(buf.getvalue()))
    print(f"cpus {os.cpu_count()} affinity {len(os.sched_getaffinity(0))}")
    for th in [int(t) for t in a.threads.split(",")]:
        with ThreadPoolExecutor(th) as ex:
            list(ex.map(lambda d: decode_image(d, 3), jp[:32]))
            t = time.perf_counter()
            list(ex.map(lambda d: decode_image(d, 3), jp))
            dt = time.perf_counter() - t
        print(f"threads {th}: {len(jp) / dt:.0f} img/s", flush=True)


if __name__ == "__main__":
    main()

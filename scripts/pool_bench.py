"""Time the Inception-v3 pooling layers alone (batch 2048, device-resident,
NHWC f32) through the engine: ms per call and effective GB/s (input read once
+ output written once). A/B knobs: TFA_POOL_GENERIC=1 (the generic window
kernel), TFA_POOL_XCD=0 (the 3x3 kernel without the XCD-contiguous block
order)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorframes_amd import engine, tf

# (name, H, W, C, k, s, padding, max)
SHAPES = [
    ("MaxPool_3a", 109, 109, 64, 3, 2, "VALID", True),
    ("MaxPool_5a", 52, 52, 192, 3, 2, "VALID", True),
    ("Mixed_6a_pool", 25, 25, 288, 3, 2, "VALID", True),
    ("Mixed_7a_pool", 12, 12, 768, 3, 2, "VALID", True),
    ("Mixed_5b_avg", 25, 25, 64, 3, 1, "SAME", False),
    ("Mixed_6b_avg", 12, 12, 192, 3, 1, "SAME", False),
    ("Mixed_7b_avg", 5, 5, 192, 3, 1, "SAME", False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = []
    for name, h, w, c, k, s, pad, is_max in SHAPES:
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, h, w, c], name="x")
            pool = tf.nn.max_pool if is_max else tf.nn.avg_pool
            tf.identity(pool(x, [1, k, k, 1], [1, s, s, 1], pad), name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn(args.batch, h, w, c, device=dev)
        y = engine.run_program(prog, [xin], dev)[0]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            y = engine.run_program(prog, [xin], dev)[0]
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        nbytes = xin.numel() * 4 + y.numel() * 4
        row = {"layer": name, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}
        out.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_ms": round(sum(r["ms"] for r in out), 4)}))


if __name__ == "__main__":
    main()

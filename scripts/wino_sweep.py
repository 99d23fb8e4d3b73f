"""Winograd F(2x2,3x3) vs the implicit-GEMM path on 3x3 stride-1 convs of one
spatial shape over a sweep of input channels C (device-resident, engine
plans, events around --iters runs). time(C) = fixed + per_stage * C / 8
separates the per-block fixed cost (prologue, epilogue) from the main loop.

    python scripts/wino_sweep.py [--batch 2048 --hw 54 --oc 192 --pad VALID --cs 16,32,64,128,256]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402


def time_conv(prog, xin, dev, iters):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        engine.run_program(prog, [xin], dev)
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        engine.run_program(prog, [xin], dev)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--hw", type=int, default=54)
    ap.add_argument("--oc", type=int, default=192)
    ap.add_argument("--pad", default="VALID")
    ap.add_argument("--cs", default="16,32,64,128,256")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    rows = []
    for c in [int(v) for v in a.cs.split(",")]:
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, a.hw, a.hw, c], name="x")
            f = tf.constant((rng.standard_normal((3, 3, c, a.oc)) * 0.05).astype(np.float32))
            tf.nn.relu(tf.nn.conv2d(x, f, [1, 1, 1, 1], a.pad), name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn((a.batch, a.hw, a.hw, c), device=dev)
        o = a.hw - 2 if a.pad == "VALID" else a.hw
        fl = 2.0 * a.batch * o * o * a.oc * 9 * c
        ms_w = time_conv(prog, xin, dev, a.iters)
        _C.set_conv_wino(False)
        ms_d = time_conv(prog, xin, dev, a.iters)
        _C.set_conv_wino(True)
        r = {"C": c, "wino_ms": ms_w, "direct_ms": ms_d, "wino_tf": fl / ms_w / 1e9, "direct_tf": fl / ms_d / 1e9}
        rows.append(r)
        print(json.dumps(r), flush=True)
    cs = np.array([r["C"] for r in rows], float)
    ms = np.array([r["wino_ms"] for r in rows])
    k, b = np.polyfit(cs / 8, ms, 1)
    print(json.dumps({"fit": "wino_ms = fixed + per_stage * C/8", "fixed_ms": b, "per_stage_ms": k}))


if __name__ == "__main__":
    main()

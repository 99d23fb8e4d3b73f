"""Chunked H2D/compute/D2H pipeline probe: relu(x @ W) over host-resident
f32[512] rows, printing wall time and the hipEvent stage times per run.

    python scripts/pipeline_probe.py [--rows 10000000] [--parts 4] [--runs 3]
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

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--parts", type=int, default=4)
ap.add_argument("--runs", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda", 0)
w = (np.random.default_rng(0).standard_normal((512, 512)) / 22.6).astype(np.float32)
g = tf.Graph()
with g.as_default():
    x = tf.placeholder(tf.float32, [None, 512], name="x")
    tf.nn.relu(tf.matmul(x, tf.constant(w)), name="y")
prog = engine.program(g.serialize(), ["y"], ["x"])
segs = []
for p in range(a.parts):
    n = (p + 1) * a.rows // a.parts - p * a.rows // a.parts
    h = _C.empty_pinned([n, 512], torch.float32)
    for s in range(0, n, 1 << 20):
        e = min(n, s + (1 << 20))
        h[s:e].copy_(torch.randn((e - s, 512), device=dev))
    segs.append([h])
torch.cuda.synchronize()
specs = [[((s[0].shape[0], 512), torch.float32)] for s in segs]
for r in range(a.runs):
    before = prog.stats()
    t0 = time.perf_counter()
    engine.run_segments_pipelined(prog, segs, specs)
    dt = time.perf_counter() - t0
    st = prog.stats()
    print(json.dumps({"run": r, "ramp": os.environ.get("TFA_PIPE_RAMP", "1"), "wall_ms": dt * 1e3,
                      "chunks": st["chunks"] - before["chunks"],
                      "h2d_ms": st["h2d_ms"] - before["h2d_ms"], "compute_ms": st["compute_ms"] - before["compute_ms"],
                      "d2h_ms": st["d2h_ms"] - before["d2h_ms"],
                      "rows_per_s": a.rows / dt}), flush=True)

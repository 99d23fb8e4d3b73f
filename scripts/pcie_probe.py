"""Host<->device staging probe: raw H2D / D2H / bidirectional copy rates from
the pinned pool, and the chunk pipeline (`run_chunked`) with an identity graph
and with the GEMM graph, to separate PCIe limits from pipeline overheads."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
res = {}
GB = 1 << 30


def bw(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


n = 1 << 28  # 1 GiB of float32
h = _C.empty_pinned([n], torch.float32)
h2 = _C.empty_pinned([n], torch.float32)
d = torch.empty(n, dtype=torch.float32, device=dev)
d2 = torch.empty(n, dtype=torch.float32, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
res["h2d_GBps"] = bw(lambda: d.copy_(h, non_blocking=True), 4 * n)
res["d2h_GBps"] = bw(lambda: h2.copy_(d, non_blocking=True), 4 * n)


def bidir():
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


res["bidir_GBps_total"] = bw(bidir, 8 * n)
pageable = torch.empty(n // 4, dtype=torch.float32)
res["h2d_pageable_GBps"] = bw(lambda: d[: n // 4].copy_(pageable), n)
del h, h2, d, d2

rows = 2_500_000
x = _C.empty_pinned([rows, 512], torch.float32)
x.normal_()
w = np.random.default_rng(0).standard_normal((512, 512)).astype(np.float32) / 22.6
for name, build in [("identity", lambda xp: tf.identity(xp, name="y")),
                    ("gemm_relu", lambda xp: tf.nn.relu(tf.matmul(xp, tf.constant(w)), name="y"))]:
    g = tf.Graph()
    with g.as_default():
        xp = tf.placeholder(tf.float32, [None, 512], name="x")
        build(xp)
    prog = engine.program(g.serialize(), ["y"], ["x"])
    out = _C.empty_pinned([rows, 512], torch.float32)
    for chunk in (32768, 131072, 524288):
        for depth in (2, 3, 4):
            prog.run_chunked([[x]], [[out]], chunk, 0, depth)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                prog.run_chunked([[x]], [[out]], chunk, 0, depth)
            dt = (time.perf_counter() - t0) / reps
            res[f"{name}_chunk{chunk}_d{depth}_GBps_each_way"] = rows * 2048 / dt / 1e9
            res[f"{name}_chunk{chunk}_d{depth}_ms"] = dt * 1e3
print(json.dumps(res, indent=1))

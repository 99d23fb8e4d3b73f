"""One f32 GEMM or Conv2D shape through the engine, repeated: the target of a
rocprofv3 --pmc pass (counters per dispatch) or a quick A/B of one tile
(TFA_GEMM_TILE=<cfg>). Prints ms and TF/s.

    python scripts/gemm_one.py gemm M N K [--iters 20]
    python scripts/gemm_one.py conv N H W C KH KW OC STRIDE PAD [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["gemm", "conv"])
    ap.add_argument("dims", nargs="+")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tb", action="store_true", help="gemm: B given as [N][K] (transpose_b)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    g = tf.Graph()
    if a.kind == "gemm":
        m, n, k = map(int, a.dims)
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, k], name="x")
            wshape = (n, k) if a.tb else (k, n)
            tf.identity(tf.matmul(x, tf.constant(rng.standard_normal(wshape).astype(np.float32)), transpose_b=a.tb),
                        name="y")
        xin = torch.randn((m, k), device=dev)
        fl = 2.0 * m * n * k
    else:
        nb, h, w, c, kh, kw, oc, s = map(int, a.dims[:8])
        pad = a.dims[8]
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, h, w, c], name="x")
            f = tf.constant((rng.standard_normal((kh, kw, c, oc)) * 0.05).astype(np.float32))
            y = tf.nn.conv2d(x, f, [1, s, s, 1], pad)
            tf.nn.relu(tf.nn.bias_add(y, tf.constant(np.zeros(oc, np.float32))), name="y")
        xin = torch.randn((nb, h, w, c), device=dev)
        oh = (h - kh) // s + 1 if pad == "VALID" else (h + s - 1) // s
        ow = (w - kw) // s + 1 if pad == "VALID" else (w + s - 1) // s
        fl = 2.0 * nb * oh * ow * oc * kh * kw * c
    prog = engine.program(g.serialize(), ["y"], ["x"])
    # warm for >= 0.3 s so the clocks have ramped before the timed loop (a
    # cold GPU times 10-20% slow on a ~10 ms loop)
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        engine.run_program(prog, [xin], dev)
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.iters):
        engine.run_program(prog, [xin], dev)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.iters
    print(json.dumps({"kind": a.kind + ("_tb" if a.tb else ""), "dims": a.dims, "tile": os.environ.get("TFA_GEMM_TILE"), "ms": ms,
                      "tflops": fl / ms / 1e9}), flush=True)


if __name__ == "__main__":
    main()

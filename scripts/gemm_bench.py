"""Kernel-level GEMM / Conv2D throughput on device-resident tensors (the f32
MFMA core of csrc/kernels/gemm.hip), timed with HIP events.

    python scripts/gemm_bench.py [--iters N] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402

GEMMS = [  # M, N, K, bias+relu
    (2_500_000, 512, 512, True),   # headline partition (BASELINE config 3)
    (262_144, 512, 512, True),
    (4096, 4096, 4096, False),
    (8192, 1024, 1024, False),
    (1_000_000, 64, 256, True),
    (100_000, 10, 100, False),
]
GEMMS_F64 = [  # M, N, K, transpose_b (K-Means shapes: points x centres^T; BASELINE config 3 in f64)
    (100_000, 10, 100, True),
    (1_000_000, 10, 100, True),
    (10_000_000, 512, 512, False),
    (4096, 4096, 4096, False),
    (262_144, 512, 512, False),
]
F64_PEAK_TF = 78.6  # MI355X FP64 matrix peak (spec)
CONVS = [  # N, H, W, C, KH, KW, OC, stride, padding (Inception-v3 @224, batch 512)
    (512, 111, 111, 32, 3, 3, 32, 1, "VALID"),
    (512, 109, 109, 32, 3, 3, 64, 1, "SAME"),
    (512, 25, 25, 192, 1, 1, 64, 1, "SAME"),
    (512, 25, 25, 48, 5, 5, 64, 1, "SAME"),
    (512, 25, 25, 64, 3, 3, 96, 1, "SAME"),
    (512, 12, 12, 768, 1, 1, 192, 1, "SAME"),
    (512, 12, 12, 128, 1, 7, 128, 1, "SAME"),
    (512, 12, 12, 160, 7, 1, 192, 1, "SAME"),
    (512, 5, 5, 1280, 1, 1, 320, 1, "SAME"),
    (512, 5, 5, 448, 3, 3, 384, 1, "SAME"),
]


def timeit(prog, ins, iters):
    engine.run_program(prog, ins, ins[0].device)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        engine.run_program(prog, ins, ins[0].device)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def vendor_time(fn, iters):
    for _ in range(2):  # library heuristics / MIOpen find on the first calls
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--f64-only", action="store_true")
    ap.add_argument("--vendor", action="store_true",
                    help="also time the same op through the ROCm libraries (torch.matmul -> hipBLASLt/rocBLAS, "
                         "F.conv2d -> MIOpen), exact f32 (no TF32/xf32), same bias+ReLU epilogue")
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    res = []
    for m, n, k, br in ([] if a.f64_only else GEMMS):
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, k], name="x")
            y = tf.matmul(x, tf.constant(rng.standard_normal((k, n)).astype(np.float32)))
            if br:
                y = tf.nn.relu(tf.nn.bias_add(y, tf.constant(rng.standard_normal(n).astype(np.float32))))
            tf.identity(y, name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn((m, k), device=dev)
        ms = timeit(prog, [xin], a.iters)
        r = {"kind": "gemm", "M": m, "N": n, "K": k, "ms": ms, "tflops": 2 * m * n * k / ms / 1e9}
        if a.vendor:
            wt = torch.randn((k, n), device=dev)
            bt = torch.randn((n,), device=dev)
            fn = (lambda: torch.relu(torch.addmm(bt, xin, wt))) if br else (lambda: xin @ wt)
            vms = vendor_time(fn, a.iters)
            r.update(vendor_ms=vms, vendor_tflops=2 * m * n * k / vms / 1e9, speedup_vs_vendor=vms / ms)
            del wt, bt
        print(json.dumps(r), flush=True)
        res.append(r)
        del xin
    for m, n, k, tb in GEMMS_F64:
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float64, [None, k], name="x")
            wv = rng.standard_normal((n, k) if tb else (k, n))
            tf.identity(tf.matmul(x, tf.constant(wv), transpose_b=tb), name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn((m, k), device=dev, dtype=torch.float64)
        ms = timeit(prog, [xin], a.iters)
        tfl = 2 * m * n * k / ms / 1e9
        r = {"kind": "gemm_f64", "M": m, "N": n, "K": k, "transpose_b": tb, "ms": ms, "tflops": tfl,
             "fraction_of_f64_peak": tfl / F64_PEAK_TF}
        print(json.dumps(r), flush=True)
        res.append(r)
        del xin
    if a.f64_only:
        CONVS.clear()
    for nb, h, w, c, kh, kw, oc, s, pad in CONVS:
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, h, w, c], name="x")
            f = tf.constant((rng.standard_normal((kh, kw, c, oc)) * 0.05).astype(np.float32))
            y = tf.nn.conv2d(x, f, [1, s, s, 1], pad)
            y = tf.nn.relu(tf.nn.bias_add(y, tf.constant(np.zeros(oc, np.float32))), name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn((nb, h, w, c), device=dev)
        ms = timeit(prog, [xin], a.iters)
        oh = (h - kh) // s + 1 if pad == "VALID" else (h + s - 1) // s
        ow = (w - kw) // s + 1 if pad == "VALID" else (w + s - 1) // s
        fl = 2 * nb * oh * ow * oc * kh * kw * c
        r = {"kind": "conv", "shape": [nb, h, w, c, kh, kw, oc, s, pad], "ms": ms, "tflops": fl / ms / 1e9}
        if a.vendor:
            import torch.nn.functional as F
            xn = xin.permute(0, 3, 1, 2)  # NHWC storage viewed as NCHW: channels_last for MIOpen
            wt = torch.randn((oc, c, kh, kw), device=dev).contiguous(memory_format=torch.channels_last)
            bt = torch.zeros((oc,), device=dev)
            if pad == "SAME":
                ph, pw = max((oh - 1) * s + kh - h, 0), max((ow - 1) * s + kw - w, 0)
                xn = F.pad(xn, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)).contiguous(
                    memory_format=torch.channels_last)
            vms = vendor_time(lambda: torch.relu(F.conv2d(xn, wt, bt, stride=s)), a.iters)
            r.update(vendor_ms=vms, vendor_tflops=fl / vms / 1e9, speedup_vs_vendor=vms / ms)
            del xn, wt, bt
        print(json.dumps(r), flush=True)
        res.append(r)
        del xin
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

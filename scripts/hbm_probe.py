"""HBM streaming ceiling vs the engine's elementwise kernel: device-to-device
copy, ATen's x + y, and the engine's Add (tfa binary kernel) on the same
1M x 128 float32 operands (config 2 shape) and on a 4x larger one.

    python scripts/hbm_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for rows in (1 << 20, 1 << 22):
        x = torch.randn((rows, 128), device=dev)
        y = torch.randn((rows, 128), device=dev)
        out = torch.empty_like(x)
        nb = x.numel() * 4
        res[f"{rows}_copy_GBps"] = 2 * nb / timeit(lambda: out.copy_(x)) / 1e9
        res[f"{rows}_aten_add_GBps"] = 3 * nb / timeit(lambda: torch.add(x, y, out=out)) / 1e9
        g = tf.Graph()
        with g.as_default():
            a = tf.placeholder(tf.float32, [None, 128], name="a")
            b = tf.placeholder(tf.float32, [None, 128], name="b")
            tf.add(a, b, name="z")
            tf.add(a, 3.0, name="z3")
        p = engine.program(g.serialize(), ["z"], ["a", "b"])
        p3 = engine.program(g.serialize(), ["z3"], ["a"])
        res[f"{rows}_tfa_add_GBps"] = 3 * nb / timeit(lambda: p.run([x, y])) / 1e9
        res[f"{rows}_tfa_add_scalar_GBps"] = 2 * nb / timeit(lambda: p3.run([x])) / 1e9
        res[f"{rows}_aten_add_scalar_GBps"] = 2 * nb / timeit(lambda: torch.add(x, 3.0, out=out)) / 1e9
    # config 4 shape: column sum of [rows, 1024] f32 (read-only stream)
    x = torch.randn((1 << 20, 1024), device=dev)
    nb = x.numel() * 4
    res["colsum_aten_GBps"] = nb / timeit(lambda: torch.sum(x, 0)) / 1e9
    g = tf.Graph()
    with g.as_default():
        a = tf.placeholder(tf.float32, [None, 1024], name="a")
        tf.reduce_sum(a, [0], name="s")
    p = engine.program(g.serialize(), ["s"], ["a"])
    res["colsum_tfa_GBps"] = nb / timeit(lambda: p.run([x])) / 1e9
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()

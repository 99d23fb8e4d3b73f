"""Per-row host overhead of a small GPU program (the per-row part of the
JPEG scoring graph: cast -> resize -> crop -> mean subtraction -> expand_dims):
time of the input copy, of a plan-cache hit and of a plan build.

    python scripts/map_rows_overhead.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402


def main():
    dev = engine.compute_device()
    g = tf.Graph()
    with g.as_default():
        im = tf.placeholder(tf.uint8, [None, None, 3], name="im")
        x = tf.image.resize_images(tf.cast(im, tf.float32), [256, 256])
        x = tf.image.central_crop_to(x, 224, 224)
        tf.expand_dims(tf.subtract(x, tf.constant(np.ones(3, np.float32))), 0, name="out")
    prog = engine.program(g.serialize(), ["out:0"], ["im"])
    rng = np.random.default_rng(0)
    imgs = [torch.from_numpy(rng.integers(0, 255, (int(h), int(w), 3), dtype=np.uint8))
            for h, w in rng.integers(180, 400, (200, 2))]
    res = {}
    # copy alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in imgs:
        t.to(dev)
    torch.cuda.synchronize()
    res["pageable_h2d_us"] = (time.perf_counter() - t0) / len(imgs) * 1e6
    # first run of every shape: plan builds
    t0 = time.perf_counter()
    for t in imgs:
        engine.run_program(prog, [t], dev)
    torch.cuda.synchronize()
    res["run_with_plan_build_us"] = (time.perf_counter() - t0) / len(imgs) * 1e6
    # second run: plan-cache hits
    t0 = time.perf_counter()
    for t in imgs:
        engine.run_program(prog, [t], dev)
    torch.cuda.synchronize()
    res["run_cached_plan_us"] = (time.perf_counter() - t0) / len(imgs) * 1e6
    # device-resident input, cached plan
    dimgs = [t.to(dev) for t in imgs]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in dimgs:
        prog.run([t])
    torch.cuda.synchronize()
    res["run_device_input_us"] = (time.perf_counter() - t0) / len(imgs) * 1e6
    # same shape every time
    t0 = time.perf_counter()
    for _ in imgs:
        prog.run([dimgs[0]])
    torch.cuda.synchronize()
    res["run_same_shape_us"] = (time.perf_counter() - t0) / len(imgs) * 1e6
    # a launch-bound chain: 40 dependent elementwise ops on a small tensor
    g2 = tf.Graph()
    with g2.as_default():
        y = tf.placeholder(tf.float32, [None, 256], name="y")
        for i in range(40):
            y = tf.tanh(y * 0.9 + 0.01 * i) if i % 2 else tf.abs(y) - 0.001
        tf.identity(y, name="chain")
    p2 = engine.program(g2.serialize(), ["chain:0"], ["y"])
    yin = torch.randn((64, 256), device=dev)
    for _ in range(20):
        p2.run([yin])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        p2.run([yin])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res["chain40_host_us"] = (t1 - t0) / 500 * 1e6
    res["chain40_total_us"] = (time.perf_counter() - t0) / 500 * 1e6
    print(os.environ.get("TFA_HIP_GRAPHS", "default"), {k: round(v, 1) for k, v in res.items()})
    print({k: v for k, v in prog.stats().items() if "graph" in k}, {k: v for k, v in p2.stats().items() if "graph" in k})


if __name__ == "__main__":
    main()

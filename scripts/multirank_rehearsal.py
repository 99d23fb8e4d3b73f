"""Multi-rank correctness rehearsal on ONE GPU: every rank drives the same
device (TFA_DIST_BACKEND=gloo, since RCCL refuses two ranks on one device),
so the device-resident SPMD paths (partition ownership, cross-rank monoid
combine, key routing for aggregate) run with real HIP kernels and are checked
against numpy on the full data.

    TFA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29513 scripts/multirank_rehearsal.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402
from tensorframes_amd.parallel import dist  # noqa: E402


def main():
    dist.init()
    rank, world = dist.rank(), dist.world_size()
    dev = engine.compute_device()
    rng = np.random.default_rng(0)
    out = {"world": world}

    # reduce_blocks Sum / Min over a device-cached frame
    x = rng.standard_normal((20_000, 64)).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=4 * world).cache_on_device(dev)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.float32, [None, 64], name="x_input")
        s = tf.reduce_sum(xi, [0], name="x")
        got = tfs.reduce_blocks(s, df)
    out["reduce_sum_err"] = float(np.abs(got - x.astype(np.float64).sum(0)).max())
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.float32, [None, 64], name="x_input")
        m = tf.reduce_min(xi, [0], name="x")
        got = tfs.reduce_blocks(m, df)
    out["reduce_min_err"] = float(np.abs(got - x.min(0)).max())

    # aggregate: per-key sums routed across ranks
    keys = rng.integers(0, 500, 20_000).astype(np.int64)
    vals = rng.standard_normal((20_000, 4))
    adf = tfs.from_columns({"key": keys, "v": vals}, num_partitions=4 * world).cache_on_device(dev)
    with tf.Graph().as_default():
        vi = tfs.block(adf, "v", tf_name="v_input")
        vs = tf.reduce_sum(vi, [0], name="v")
        res = tfs.aggregate(vs, adf.groupBy("key")).collect()
    want = {}
    for k_, v_ in zip(keys, vals):
        want[int(k_)] = want.get(int(k_), 0) + v_
    out["aggregate_groups"] = len(res)
    out["aggregate_err"] = max(float(np.abs(np.array(r["v"]) - want[int(r["key"])]).max()) for r in res)

    # K-Means (in-graph variant) on the device-cached frame, 3 iterations
    pts = rng.uniform(0, 1, (10_000, 20))
    kdf = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4 * world)).cache_on_device(dev)
    c0 = np.random.default_rng(1).standard_normal((5, 20))
    c, _ = kmeans.kmeans(kdf, c0, num_iters=3)
    cn = c0
    for _ in range(3):  # the in-graph variant's update: sums / (counts + 1e-7)
        d = (pts ** 2).sum(1)[:, None] + (cn ** 2).sum(1)[None, :] - 2 * pts @ cn.T
        idx = d.argmin(1)
        sums = np.zeros_like(cn)
        np.add.at(sums, idx, pts)
        cn = sums / (np.bincount(idx, minlength=cn.shape[0]) + 1e-7)[:, None]
    out["kmeans_center_err"] = float(np.abs(c - cn).max())
    ok = (out["reduce_sum_err"] < 1e-2 and out["reduce_min_err"] == 0.0 and out["aggregate_groups"] == 500
          and out["aggregate_err"] < 1e-9 and out["kmeans_center_err"] < 1e-6)
    out["ok"] = bool(ok)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

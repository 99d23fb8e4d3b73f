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
    from tensorframes_amd._native import _C
    pool0 = _C.device_pool_stats()
    torch0 = torch.cuda.memory_stats(dev).get("allocation.all.allocated", 0)

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

    # Prod / Max reducers (identity fills), groupBy().count(), long string
    # keys (hashed, routed with their bytes), repartition of a device frame
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.float32, [None, 64], name="x_input")
        got = tfs.reduce_blocks(tf.reduce_max(xi, [0], name="x"), df)
    out["reduce_max_err"] = float(np.abs(got - x.max(0)).max())
    cnt = {int(r["key"]): int(r["count"]) for r in adf.groupBy("key").count().collect()}
    out["count_err"] = int(sum(abs(cnt.get(k_, 0) - int(c_)) for k_, c_ in
                               zip(*np.unique(keys, return_counts=True))))
    skeys = np.array([f"user-{i % 97:03d}" * (1 + i % 3) for i in range(6000)])
    sv = rng.standard_normal(6000)
    sdf = tfs.from_columns({"k": skeys, "x": sv}, num_partitions=2 * world)
    with tf.Graph().as_default():
        si = tf.placeholder(tf.double, [None], name="x_input")
        srows = tfs.aggregate(tf.reduce_sum(si, [0], name="x"), sdf.groupBy("k")).collect()
    swant = {}
    for k_, v_ in zip(skeys, sv):
        swant[k_] = swant.get(k_, 0.0) + v_
    out["string_groups"] = len(srows)
    out["string_err"] = max(abs(r.x - swant[r.k]) for r in srows) if srows else 0.0
    rp = adf.repartition(3 * world)
    out["repartition_rows"] = int(rp.count())

    pool1 = _C.device_pool_stats()
    torch1 = torch.cuda.memory_stats(dev).get("allocation.all.allocated", 0)
    stats = torch.tensor([pool1["fallbacks"] - pool0["fallbacks"], pool1["allocs"] - pool0["allocs"],
                          torch1 - torch0], dtype=torch.int64)
    dist.all_reduce_host_(stats, "Max")
    out["pool_fallbacks"], out["pool_allocs"], out["framework_allocs"] = (int(v) for v in stats.tolist())
    ok = (out["reduce_sum_err"] < 1e-2 and out["reduce_min_err"] == 0.0 and out["aggregate_groups"] == 500
          and out["aggregate_err"] < 1e-9 and out["kmeans_center_err"] < 1e-6 and out["reduce_max_err"] == 0.0
          and out["count_err"] == 0 and out["string_groups"] == len(swant) and out["string_err"] < 1e-9
          and out["repartition_rows"] == 20_000 and out["pool_fallbacks"] == 0 and out["pool_allocs"] > 0)
    out["ok"] = bool(ok)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

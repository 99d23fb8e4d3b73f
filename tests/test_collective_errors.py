"""Data-dependent failures inside SPMD operators are collective (CPU, world 4
and 8, the engine's shared-memory data path): a fault injected on ONE rank in
reduce_blocks, reduce_rows, aggregate or an eager map_blocks makes every rank
raise within seconds (parallel/dist.agreed) instead of the other ranks waiting
in the next collective for `collective_timeout_s`; a string-key hash
collision that only the owning rank detects makes every rank redo the
aggregation on exact key words, with exact results. Also: half / bfloat16 /
bool host all-reduces (which the shared-memory communicator does not fold)
still work at world 2. Reference: Spark fails the whole job on a task failure
(DebugRowOps.scala:500, :524-525, :576)."""
import json
import os
import socket
import sys
import time

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1", TFA_SHM_COLLECTIVES="1", TFA_DEVICE="cpu",
                      TFA_COLLECTIVE_TIMEOUT_S="60")
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from tensorframes_amd.parallel import dist
    assert dist.init(backend="gloo")


def _timed(fn):
    t0 = time.time()
    try:
        fn()
        return {"err": None, "secs": time.time() - t0}
    except Exception as e:  # noqa: BLE001
        return {"err": type(e).__name__, "msg": str(e)[:200], "secs": time.time() - t0}


def _fail_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    import numpy as np

    import tensorframes_amd as tfs
    from tensorframes_amd import Row, tf
    from tensorframes_amd.utils import faults
    bad = 1
    data = [Row(key=str(i % 3), x=float(i)) for i in range(40)]
    df = tfs.analyze(tfs.create_dataframe(data, num_partitions=world))
    res = {}
    with faults.inject("reduce_blocks", rank=bad, times=1), tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["reduce_blocks"] = _timed(lambda: tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df.select("x")))
    with faults.inject("reduce_rows", rank=bad, times=1), tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x2 = tf.placeholder(tf.double, shape=[], name="x_2")
        res["reduce_rows"] = _timed(lambda: tfs.reduce_rows(tf.add(x1, x2, name="x"), df.select("x")))
    with faults.inject("aggregate", rank=bad, times=1), tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.select("key", "x").groupBy("key"))
        res["aggregate"] = _timed(agg.collect)
    with faults.inject("map_blocks", rank=bad, times=1), tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        out = tfs.map_blocks(tf.multiply(x, 2.0, name="z"), df.select("x"))
        res["map_blocks_collect"] = _timed(out.collect)
    # afterwards the job is healthy again: every rank runs the next collective
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["after"] = float(tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df.select("x")))
    res["expected_after"] = float(np.sum(np.arange(40)))
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)


@pytest.mark.parametrize("world", [4, 8])
def test_one_rank_failure_raises_on_every_rank(world, tmp_path):
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        o = json.load(open(tmp_path / f"r{r}.json"))
        for site in ("reduce_blocks", "reduce_rows", "aggregate", "map_blocks_collect"):
            got = o[site]
            assert got["err"] is not None, (r, site, got)
            assert got["secs"] < 5.0, (r, site, got)
            if r == 1:
                assert got["err"] == "InjectedFault", (site, got)
            else:
                assert got["err"] == "RemoteRankError" and "rank 1" in got["msg"], (r, site, got)
        assert o["after"] == o["expected_after"]


def _collision_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    import numpy as np

    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.ops import groupby as G
    from tensorframes_amd.utils.logging import metrics
    real = G.string_key_hashed

    def colliding(col, dev):  # every long key gets the same hash tag
        w0, t = real(col, dev)
        return [w0, torch.where(t >= G.HASH_TAG_MIN, torch.full_like(t, G.HASH_TAG_MIN), t)]
    G.string_key_hashed = colliding
    keys = np.array(["collide_" + "a" * 20, "collide_" + "b" * 20, "short", "other_key_long_enough"])[
        np.arange(400) % 4]
    x = np.arange(400, dtype=np.float64)
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=world)
    metrics.reset()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        rows = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k")).collect()
    want = {k: float(x[keys == k].sum()) for k in set(keys.tolist())}
    got = {r.k: r.x for r in rows}
    snap = metrics.snapshot()
    with open(os.path.join(outdir, f"c{rank}.json"), "w") as f:
        json.dump({"ok": got == want, "got": got, "collisions": snap.get("aggregate_string_key_collisions", 0)}, f)


def test_collision_on_one_rank_falls_back_on_all(tmp_path):
    world = 4
    mp.spawn(_collision_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        o = json.load(open(tmp_path / f"c{r}.json"))
        assert o["ok"], o
        assert o["collisions"] == 1, o  # every rank took the exact-width rerun


def _dtype_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    from tensorframes_amd.parallel import dist
    res = {}
    for name, dt in (("f16", torch.float16), ("bf16", torch.bfloat16)):
        t = torch.full((5,), 1.5 * (rank + 1), dtype=dt)
        dist.all_reduce_(t, "Sum")
        res[name] = t.float().tolist()
    b = torch.tensor([rank == 0, False, True])
    dist.all_reduce_host_(b, "Max")
    res["bool"] = b.tolist()
    with open(os.path.join(outdir, f"d{rank}.json"), "w") as f:
        json.dump(res, f)


def test_half_bf16_bool_all_reduce_use_gloo(tmp_path):
    mp.spawn(_dtype_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        o = json.load(open(tmp_path / f"d{r}.json"))
        assert o["f16"] == [4.5] * 5 and o["bf16"] == [4.5] * 5
        assert o["bool"] == [True, False, True]

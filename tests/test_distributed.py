"""Multi-process (SPMD) execution on the CPU at world size 2, 3, 4 and 8:
partitions pinned to ranks, collect/count gathers, reduce_blocks /
reduce_rows cross-rank combine (all-reduce for monoids, all-gather + one
graph run otherwise), aggregate's key shuffle (all-to-all), repartition.

The data path runs through the engine's own shared-memory communicator
(csrc/comm ShmComm, parallel/comm.init_host): the collective counters must
show its calls and no gloo tensor collective or pickled object exchange on
the reduce / aggregate paths (gloo is only the bootstrap). World 2 also runs
with the shared-memory path off (the gloo fallback). Reference cross-partition
points: DebugRowOps.scala:500, :524-525, :576, :732-750."""
import json
import os
import socket
import sys

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


def _worker(rank, world, port, outdir, device="cpu", shm=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="1",
                      TFA_SHM_COLLECTIVES="1" if shm else "0")
    if device == "cpu":
        os.environ["TFA_DEVICE"] = "cpu"
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    import numpy as np

    import tensorframes_amd as tfs
    from tensorframes_amd import Row, tf
    from tensorframes_amd.parallel import dist

    assert dist.init(backend="gloo")
    from tensorframes_amd import engine
    res = {"device": engine.compute_device().type}
    data = [Row(key=str(i % 3), k=i % 4, x=float(i), v=[float(i), float(2 * i)]) for i in range(20)]
    df = tfs.analyze(tfs.create_dataframe(data, num_partitions=5))
    res["local_parts"] = sorted(df.local_blocks())
    res["count"] = df.count()
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        out = tfs.map_blocks(tf.multiply(x, 2.0, name="z"), df)
        res["z"] = [r.z for r in out.collect()]
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["sum"] = tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df.select("x"))
    with tf.Graph().as_default():
        vi = tf.placeholder(tf.double, shape=[None, 2], name="v_input")
        res["vmax"] = tfs.reduce_blocks(tf.reduce_max(vi, [0], name="v"), df.select("v")).tolist()
    with tf.Graph().as_default():
        # generic (non-monoid) associative graph: sum of squares of... identity of the sum
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["gen"] = tfs.reduce_blocks(tf.identity(tf.reduce_sum(xi, [0]), name="x"), df.select("x"))
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x2 = tf.placeholder(tf.double, shape=[], name="x_2")
        res["rows"] = tfs.reduce_rows(tf.add(x1, x2, name="x"), df.select("x"))
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.select("key", "x").groupBy("key"))
        res["agg"] = sorted([list(r) for r in agg.collect()])
    with tf.Graph().as_default():
        # integer keys + vector cells: both shuffle as tensors (all_to_all_single)
        vi = tf.placeholder(tf.double, shape=[None, 2], name="v_input")
        agg = tfs.aggregate(tf.reduce_sum(vi, [0], name="v"), df.select("k", "v").groupBy("k"))
        res["agg_int"] = sorted([[r.k, list(r.v)] for r in agg.collect()])
    with tf.Graph().as_default():
        # not a recognised monoid: rows shuffle, then one graph run per key
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.identity(tf.reduce_sum(xi * xi, [0]), name="x"), df.select("k", "x").groupBy("k"))
        res["agg_gen"] = sorted([[r.k, r.x] for r in agg.collect()])
    with tf.Graph().as_default():
        # one key: every other rank receives nothing from the shuffle
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        one = tfs.create_dataframe([Row(c="a", x=float(i)) for i in range(20)], num_partitions=5)
        agg = tfs.aggregate(tf.reduce_min(xi, [0], name="x"), one.groupBy("c"))
        res["agg_one"] = [list(r) for r in agg.collect()]
    # int32 keys + float64 values through the packed-record shuffle, with
    # fewer groups than ranks (most ranks receive 0 or 1 rows), non-monoid
    import numpy as _np
    kk = _np.array([i % 2 for i in range(12)], dtype=_np.int32)
    xx = _np.arange(12, dtype=_np.float64)
    few = tfs.from_columns({"k": kk, "x": xx}, num_partitions=6)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.identity(tf.reduce_max(xi, [0]) * 2.0, name="x"), few.groupBy("k"))
        res["agg_few"] = sorted([[int(r.k), float(r.x)] for r in agg.collect()])
    # reductions make no host-object (pickled gloo) exchange; ranks without
    # data contribute identities (1 partition: only rank 0 has rows), also
    # when the output shape is only known at run time (unanalysed [?,?] column)
    from tensorframes_amd.utils.logging import metrics as _m
    snap0 = _m.snapshot()
    ago0 = snap0.get("collective_all_gather_object", 0)
    gloo0 = {k: snap0.get(k, 0) for k in ("collective_all_reduce", "collective_all_gather", "collective_all_to_all",
                                          "collective_all_to_all_objects")}
    one_part = tfs.create_dataframe([Row(x=float(i), v=[float(i), 1.0]) for i in range(7)], num_partitions=1)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["sum_one_part"] = tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), one_part.select("x"))
    with tf.Graph().as_default():
        vi = tf.placeholder(tf.double, shape=[None, None], name="v_input")
        res["vmin_one_part"] = tfs.reduce_blocks(tf.reduce_min(vi, [0], name="v"), one_part.select("v")).tolist()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        res["gen_one_part"] = tfs.reduce_blocks(tf.identity(tf.reduce_max(xi, [0]), name="x"), one_part.select("x"))
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.select("key", "x").groupBy("key"))
        res["agg2"] = sorted([list(r) for r in agg.collect()])
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, shape=[None], name="x_input")
        agg = tfs.aggregate(tf.identity(tf.reduce_sum(xi * xi, [0]), name="x"), df.select("key", "x").groupBy("key"))
        res["agg_gen_str"] = sorted([list(r) for r in agg.collect()])
    snap1 = _m.snapshot()
    res["ago_delta"] = snap1.get("collective_all_gather_object", 0) - ago0
    res["gloo_delta"] = {k: snap1.get(k, 0) - v for k, v in gloo0.items()}
    res["repart"] = [r.x for r in df.repartition(4).select("x").collect()]
    # checkpoint: every rank writes its own partitions, reads them back
    ck = os.path.join(outdir, "ck")
    back = tfs.read_checkpoint(df.write_checkpoint(ck))
    res["ck_parts"] = sorted(back.local_blocks())
    res["ck_x"] = [r.x for r in back.collect()]
    # parquet: each rank writes its partitions, reads its row groups back
    pq_dir = os.path.join(outdir, "pq")
    back_pq = tfs.read_parquet(df.select("x", "v").write_parquet(pq_dir), num_partitions=5)
    res["pq_x"] = [r.x for r in back_pq.collect()]
    res["pq_parts"] = sorted(back_pq.local_blocks())
    # a fault injected on rank 1 only is retried locally; results stay consistent
    from tensorframes_amd.utils import faults
    tfs.set_config(task_retries=1)
    with faults.inject("map_blocks", rank=1, times=1):
        with tf.Graph().as_default():
            x = tf.placeholder(tf.double, shape=[None], name="x")
            res["retry_z"] = [r.z for r in tfs.map_blocks(tf.add(x, 1.0, name="z"), df.select("x")).collect()]
    from tensorframes_amd.utils.logging import metrics
    res["coll"] = {k: v for k, v in metrics.snapshot().items() if k.startswith("collective_")}
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.shutdown()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_spmd_world(world, tmp_path):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    _check_results(tmp_path, world, "cpu", shm=True)


def test_spmd_world_gloo_fallback(tmp_path):
    """The same program with the shared-memory path off: host collectives over gloo."""
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), "cpu", False), nprocs=2, join=True)
    _check_results(tmp_path, 2, "cpu", shm=False)


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() == 0, reason="needs a GPU")
def test_spmd_two_ranks_share_one_gpu(tmp_path):
    """The same SPMD program with both ranks computing on the GPU (gloo
    rehearsal: device tensors are staged through the host for collectives,
    since RCCL cannot put two ranks on one GPU)."""
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), "gpu"), nprocs=2, join=True)
    _check_results(tmp_path, 2, "cuda")


def _check_results(tmp_path, world, device, shm=False):
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    assert all(o["device"] == device for o in outs)
    for o in outs:  # collectives are counted (metrics) on every rank
        c = o["coll"]
        reduces = sum(c.get(k, 0) for k in ("collective_all_reduce", "collective_oneshot_all_reduce",
                                             "collective_rccl_all_reduce", "collective_shm_all_reduce"))
        a2a = sum(c.get(k, 0) for k in ("collective_all_to_all", "collective_rccl_all_to_all",
                                         "collective_shm_all_to_all"))
        assert a2a >= 1 and reduces >= 1
        assert c["collective_bytes"] > 0
        if shm:
            # the engine's communicator carried the data: no gloo tensor
            # collective and no pickled exchange on the reduce/aggregate paths
            assert c.get("collective_shm_all_reduce", 0) >= 1 and c.get("collective_shm_all_to_all", 0) >= 1
            assert all(v == 0 for v in o["gloo_delta"].values()), o["gloo_delta"]
    xs = [float(i) for i in range(20)]
    parts = sorted(p for o in outs for p in o["local_parts"])
    assert parts == [0, 1, 2, 3, 4]
    for r, o in enumerate(outs):
        assert o["local_parts"] == [p for p in range(5) if p % world == r]
        assert o["count"] == 20
        assert o["z"] == [2 * x for x in xs]
        assert o["sum"] == sum(xs) == o["gen"] == o["rows"]
        assert o["vmax"] == [19.0, 38.0]
        want = sorted([[k, sum(x for x in xs if str(int(x) % 3) == k)] for k in ("0", "1", "2")])
        assert o["agg"] == want
        assert o["agg_int"] == [[k, [sum(x for x in xs if int(x) % 4 == k), 2 * sum(x for x in xs if int(x) % 4 == k)]]
                                for k in range(4)]
        assert o["agg_gen"] == [[k, sum(x * x for x in xs if int(x) % 4 == k)] for k in range(4)]
        assert o["agg_one"] == [["a", 0.0]]
        assert o["agg2"] == want
        assert o["agg_gen_str"] == sorted([[k, sum(x * x for x in xs if str(int(x) % 3) == k)] for k in ("0", "1", "2")])
        assert o["agg_few"] == [[0, 20.0], [1, 22.0]]
        assert o["sum_one_part"] == 21.0 and o["vmin_one_part"] == [0.0, 1.0] and o["gen_one_part"] == 6.0
        assert o["ago_delta"] == 0
        assert o["repart"] == xs
        assert o["ck_parts"] == o["local_parts"] and o["ck_x"] == xs
        assert o["retry_z"] == [x + 1.0 for x in xs]
        assert o["pq_x"] == xs and o["pq_parts"] == o["local_parts"]


def test_parse_cpulist_and_bind_numa_noop_without_gpu():
    from tensorframes_amd.parallel import dist as D
    assert D._parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert D._parse_cpulist("") == []
    assert D.bind_numa() == []  # no GPU here: nothing to bind

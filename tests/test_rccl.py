"""RCCL on an executed path: a world-size-1 NCCL (= RCCL) process group with
`force_collectives`, so reduce_blocks / reduce_rows / aggregate issue exactly
the device collectives an 8-rank job issues, on the one GPU of the test box.

Reference counterparts: RDD.reduce of the partials (src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500,524-525)
and the groupBy shuffle (DebugRowOps.scala:576)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_group(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import torch.distributed as tdist

    from tensorframes_amd.config import config
    from tensorframes_amd.parallel import dist
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("TFA_DEVICE", "cuda")
    old = config.force_collectives
    assert not tdist.is_initialized()
    try:
        assert dist.init(backend="nccl", force=True)
        assert tdist.get_backend() == "nccl" and tdist.get_world_size() == 1
        assert dist.gpu_collectives()
        from tensorframes_amd.parallel import comm
        # the engine communicator is built once, collectively (its one-time
        # setup exchanges device ids and IPC handles over the host group)
        assert comm.get() is not None
        yield dist
    finally:
        dist.shutdown()
        config.force_collectives = old
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
            monkeypatch.delenv(k, raising=False)


def _delta(before, after, key):
    return after.get(key, 0) - before.get(key, 0)


def test_reduce_blocks_runs_one_rccl_allreduce_per_op(rccl_group):
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.utils.logging import metrics
    rng = np.random.default_rng(0)
    x = rng.standard_normal((5000, 64)).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=4).cache_on_device("cuda:0")
    for op, fn, ref in (("Sum", tf.reduce_sum, x.astype(np.float64).sum(0)),
                        ("Min", tf.reduce_min, x.min(0)), ("Max", tf.reduce_max, x.max(0))):
        before = metrics.snapshot()
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.float32, [None, 64], name="x_input")
            got = tfs.reduce_blocks(fn(xi, [0], name="x"), df)
        after = metrics.snapshot()
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-3)
        # one device all-reduce, through the engine's own communicator: the
        # partial (65 floats) takes the one-shot IPC path, not torch's RCCL
        assert _delta(before, after, "collective_oneshot_all_reduce") == 1, op
        assert _delta(before, after, "collective_all_reduce") == 0, op
        assert _delta(before, after, "collective_all_gather_object") == 0, op
    assert rccl_group.collective_device_ms() > 0


def test_reduce_blocks_two_fetches_share_one_allreduce(rccl_group):
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.utils.logging import metrics
    a = np.arange(1000, dtype=np.float64)
    df = tfs.from_columns({"a": a, "b": 2 * a}, num_partitions=3).cache_on_device("cuda:0")
    before = metrics.snapshot()
    with tf.Graph().as_default():
        ai = tf.placeholder(tf.double, [None], name="a_input")
        bi = tf.placeholder(tf.double, [None], name="b_input")
        ra, rb = tfs.reduce_blocks([tf.reduce_sum(ai, [0], name="a"), tf.reduce_sum(bi, [0], name="b")], df)
    after = metrics.snapshot()
    assert ra == a.sum() and rb == 2 * a.sum()
    assert _delta(before, after, "collective_oneshot_all_reduce") == 1


def test_reduce_rows_and_generic_reduce_over_rccl(rccl_group):
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.utils.logging import metrics
    df = tfs.create_dataframe([tfs.Row(x=float(i)) for i in range(100)], num_partitions=4)
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, [], name="x_1")
        x2 = tf.placeholder(tf.double, [], name="x_2")
        assert tfs.reduce_rows(tf.add(x1, x2, name="x"), df) == 4950.0
    before = metrics.snapshot()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        # not a recognised monoid: per-rank partial, all-gathered, graph run once more
        got = tfs.reduce_blocks(tf.identity(tf.reduce_sum(xi, [0]), name="x"), df)
    after = metrics.snapshot()
    assert got == 4950.0
    assert _delta(before, after, "collective_rccl_all_gather") >= 1  # the engine's RCCL communicator
    assert _delta(before, after, "collective_all_gather_object") == 0


def test_aggregate_shuffle_over_rccl(rccl_group):
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.utils.logging import metrics
    n = 20000
    keys = (np.arange(n) % 37).astype(np.int64)
    x = np.random.default_rng(1).standard_normal((n, 8))
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=4).cache_on_device("cuda:0")
    before = metrics.snapshot()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None, 8], name="x_input")
        out = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k"))
        rows = sorted(out.collect(), key=lambda r: r.k)
    after = metrics.snapshot()
    assert _delta(before, after, "collective_rccl_all_to_all") >= 1  # grouped send/recv of the engine's comm
    assert len(rows) == 37
    for r in rows:
        np.testing.assert_allclose(r.x, x[keys == r.k].sum(0), rtol=1e-10, atol=1e-9)

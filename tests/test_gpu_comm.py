"""The engine communicator on the GPU (csrc/comm, kernels/oneshot.hip):

* RcclComm — the engine's own RCCL communicator (ncclCommInitRank) at world
  size 1: all_reduce / all_gather / all_to_all_v / broadcast on the current
  stream;
* OneShotComm — the single-hop IPC all-reduce at world size 1, and with two
  ranks (processes) sharing the one GPU: every dtype and op against numpy,
  payloads up to the 64 KB cap, enough calls to cycle both buffer slots.

The N = 2/4/8 contract runs on FakeComm in tests/test_comm.py. Reference: the
partial combine and the groupBy shuffle of
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500,524-525,576,732-750."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

OPS = {"Sum": np.add.reduce, "Min": np.minimum.reduce, "Max": np.maximum.reduce, "Prod": np.multiply.reduce}
DTYPES = [torch.float32, torch.float64, torch.int32, torch.int64]


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_rccl_comm_world_one():
    _need_gpu()
    from tensorframes_amd._native import _C
    c = _C.RcclComm(_C.rccl_unique_id(), 0, 1, 0)
    assert c.kind == "rccl" and c.rank == 0 and c.size == 1
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    assert torch.equal(c.all_reduce(x.clone(), "Sum"), x)
    g = c.all_gather(x)
    assert g.shape == (1, 1000) and torch.equal(g[0], x)
    rows = torch.arange(30, dtype=torch.int64, device="cuda").reshape(10, 3)
    assert torch.equal(c.all_to_all_v(rows, [10], [10]), rows)
    assert torch.equal(c.broadcast(x.clone(), 0), x)
    c.barrier()
    assert c.async_error() == ""
    assert c.calls >= 5


@pytest.mark.parametrize("dtype", DTYPES)
def test_oneshot_world_one(dtype):
    _need_gpu()
    from tensorframes_amd._native import _C
    o = _C.OneShotComm(0, 1, 0)
    o.open([o.ipc_handle()])
    assert o.ready
    for op in OPS:
        x = (torch.arange(257, device="cuda") % 7 + 1).to(dtype)
        y = o.all_reduce(x.clone(), op)
        torch.cuda.synchronize()
        assert torch.equal(y, x), op
    o.check()
    with pytest.raises(Exception):
        o.all_reduce(torch.zeros(_C.OneShotComm.max_bytes() // 4 + 1, device="cuda"), "Sum")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oneshot_worker(rank, world, port, outdir):
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as tdist

    from tensorframes_amd._native import _C
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    o = _C.OneShotComm(rank, world, 0)
    hs = [None] * world
    tdist.all_gather_object(hs, o.ipc_handle())
    o.open(hs)
    rng = np.random.default_rng(1234)
    res = {"bad": []}
    # the same sequence on both ranks: sizes up to the 64 KB cap, every dtype
    # and op, more calls than slots
    for it in range(24):
        dt = DTYPES[it % 4]
        op = list(OPS)[(it // 4) % 4]
        n = [1, 100, 1025, 16384 if dt in (torch.float32, torch.int32) else 8192][it % 4]
        vals = [rng.integers(1, 4, size=n) for _ in range(world)]
        x = torch.from_numpy(vals[rank]).to(dt).cuda()
        y = o.all_reduce(x, op).cpu().numpy().astype(np.float64)
        want = OPS[op](np.stack(vals).astype(np.float64), axis=0)
        if not np.allclose(y, want, rtol=1e-5):
            res["bad"].append([it, str(dt), op, n])
    torch.cuda.synchronize()
    o.check()
    res["calls"] = o.calls
    with open(os.path.join(outdir, f"os{rank}.json"), "w") as f:
        json.dump(res, f)
    tdist.barrier()
    tdist.destroy_process_group()


def test_oneshot_two_ranks_share_one_gpu(tmp_path):
    """Two processes on the one GPU: the flags and partials cross process
    boundaries through the IPC mappings, as they cross GPUs on a node."""
    _need_gpu()
    import json

    import torch.multiprocessing as mp
    mp.spawn(_oneshot_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = json.load(open(tmp_path / f"os{r}.json"))
        assert res["bad"] == [] and res["calls"] == 24, res


def test_engine_comm_serves_reduce_blocks_under_rccl_group(monkeypatch):
    """A world-size-1 RCCL process group with force_collectives: the
    reduce_blocks combine runs on the engine's one-shot path."""
    _need_gpu()
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.config import config
    from tensorframes_amd.parallel import comm, dist
    from tensorframes_amd.utils.logging import metrics
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    old = config.force_collectives
    try:
        assert dist.init(backend="nccl", force=True)
        ec = comm.get()
        assert ec is not None and ec.kinds == ["oneshot", "rccl"]
        x = np.random.default_rng(0).standard_normal((4096, 1024)).astype(np.float32)
        df = tfs.from_columns({"x": x}, num_partitions=4).cache_on_device("cuda:0")
        before = metrics.snapshot().get("collective_oneshot_all_reduce", 0)
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.float32, [None, 1024], name="x_input")
            got = tfs.reduce_blocks(tf.reduce_sum(xi, [0], name="x"), df)
        np.testing.assert_allclose(got, x.astype(np.float64).sum(0), rtol=1e-4, atol=1e-2)
        assert metrics.snapshot().get("collective_oneshot_all_reduce", 0) - before == 1
    finally:
        dist.shutdown()
        config.force_collectives = old

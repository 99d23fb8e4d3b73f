"""The engine communicator on the GPU (csrc/comm, kernels/oneshot.hip):

* RcclComm — the engine's own RCCL communicator (ncclCommInitRank) at world
  size 1: all_reduce / all_gather / all_to_all_v / broadcast on the current
  stream;
* OneShotComm — the single-hop IPC all-reduce at world size 1, and with two
  ranks (processes) sharing the one GPU: every dtype and op against numpy,
  payloads up to the 64 KB cap, enough calls to cycle both buffer slots.

Failure detection: a collective queued behind a stalled stream
(kernels device_stall, a bounded spin) makes RcclComm.wait() raise
CollectiveError at the timeout instead of hanging; a process stuck in an
unbounded synchronisation is ended by the watchdog with status 76. The
one-shot path's start-up self-test runs at world 1 and with two ranks on the
GPU, and a forced failure switches every rank to RCCL.

The N = 2/4/8 contract runs on FakeComm in tests/test_comm.py and on the
shared-memory communicator in tests/test_shm_comm.py. Reference: the
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
    from tensorframes_amd.parallel import comm as _comm
    res = {"bad": [], "selftest": _comm._oneshot_self_test(o, rank, world, 0), "alloc": o.alloc_kind}
    rng = np.random.default_rng(1234)
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
        assert res["selftest"] is None, res  # the start-up self-test passes across processes
        assert res["bad"] == [] and res["calls"] == 24 + 6, res


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


def test_oneshot_buffer_is_uncached():
    """The flag/slot buffer must not be L2-cacheable (peers write it over xGMI)."""
    _need_gpu()
    from tensorframes_amd._native import _C
    o = _C.OneShotComm(0, 1, 0)
    assert o.alloc_kind in ("uncached", "fine-grained"), o.alloc_kind


def _forced_world(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)


def test_oneshot_self_test_and_forced_fallback(monkeypatch):
    """world 1 (RCCL group, force_collectives): the self-test enables the
    one-shot path; TFA_ONESHOT_SELFTEST_FAIL=1 makes every rank use RCCL."""
    _need_gpu()
    from tensorframes_amd.config import config
    from tensorframes_amd.parallel import comm, dist
    from tensorframes_amd.utils.logging import metrics
    _forced_world(monkeypatch)
    old = config.force_collectives
    try:
        assert dist.init(backend="nccl", force=True)
        ok0 = metrics.snapshot().get("oneshot_selftest_ok", 0)
        ec = comm.get()
        assert ec.kinds == ["oneshot", "rccl"]
        assert metrics.snapshot().get("oneshot_selftest_ok", 0) == ok0 + 1
        dist.shutdown()
        monkeypatch.setenv("TFA_ONESHOT_SELFTEST_FAIL", "1")
        monkeypatch.delenv("MASTER_PORT", raising=False)
        assert dist.init(backend="nccl", force=True)
        ec = comm.get()
        assert ec.kinds == ["rccl"]
        t = torch.ones(16, device="cuda")
        ec.all_reduce_(t)  # small payload now on RCCL
        ec.wait()
        assert t.tolist() == [1.0] * 16
    finally:
        dist.shutdown()
        config.force_collectives = old


def test_rccl_queued_collective_does_not_time_out_behind_compute():
    """A collective queued behind 2 s of other work on its stream is NOT timed
    out at 0.5 s: its clock starts when it starts (a start event before it),
    so a backed-up stream never trips the watchdog of a healthy rank."""
    _need_gpu()
    import time

    from tensorframes_amd._native import _C
    c = _C.RcclComm(_C.rccl_unique_id(), 0, 1, 0)
    c.set_timeout(0.5, False)
    x = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    _C.device_stall(2.0)
    c.all_reduce(x, "Sum")
    t0 = time.time()
    c.wait()
    assert time.time() - t0 > 1.0 and not c.failed and c.inflight == 0


def test_rccl_wait_times_out_and_aborts_a_started_collective():
    """A collective that started and does not finish (test stall inside it)
    raises CollectiveError at the 0.5 s timeout; the communicator is aborted
    (ncclCommAbort releases a collective kernel waiting for a peer), so a later
    device synchronisation returns in bounded time, and it refuses new
    collectives."""
    _need_gpu()
    import time

    from tensorframes_amd._native import _C
    c = _C.RcclComm(_C.rccl_unique_id(), 0, 1, 0)
    c.set_timeout(0.5, False)
    x = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    c.set_test_stall(3.0)
    c.all_reduce(x, "Sum")
    t0 = time.time()
    with pytest.raises(_C.CollectiveError, match="timed out"):
        c.wait()
    waited = time.time() - t0
    assert waited < 3.0, waited
    t1 = time.time()
    torch.cuda.synchronize()
    assert time.time() - t1 < 10.0
    assert c.failed and c.async_error() == "aborted"
    with pytest.raises(_C.CollectiveError):
        c.all_reduce(x, "Sum")
    # a healthy communicator: wait() returns once the work is done
    c2 = _C.RcclComm(_C.rccl_unique_id(), 0, 1, 0)
    c2.set_timeout(5.0, False)
    c2.all_reduce(x, "Sum")
    c2.wait()
    assert c2.inflight == 0 and not c2.failed


def test_rccl_watchdog_ends_a_stuck_process(tmp_path):
    """The main thread blocks in an unbounded synchronisation on a collective
    that started and does not finish: the watchdog aborts the communicator
    and exits with 76."""
    _need_gpu()
    import subprocess
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, time, torch; sys.path.insert(0, %r)\n"
        "from tensorframes_amd._native import _C\n"
        "c = _C.RcclComm(_C.rccl_unique_id(), 0, 1, 0)\n"
        "c.set_timeout(0.3, True)\n"
        "x = torch.ones(1 << 20, device='cuda'); torch.cuda.synchronize()\n"
        "print('T0', time.time(), flush=True)\n"
        "c.set_test_stall(12.0)\n"
        "c.all_reduce(x, 'Sum')\n"
        "torch.cuda.synchronize()\n"
        "print('NOT REACHED')\n" % repo)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    end = time.time()
    assert p.returncode == 76, (p.returncode, p.stderr[-2000:])
    assert "NOT REACHED" not in p.stdout and "aborting the RCCL communicator" in p.stderr
    t0 = float(p.stdout.split("T0")[1].split()[0])
    assert end - t0 < 9.0, end - t0  # ended by the watchdog, not by the 12 s stall finishing

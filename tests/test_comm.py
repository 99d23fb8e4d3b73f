"""The engine communicator's collective contract (csrc/comm/comm.h), run on
FakeComm: N in-process ranks (threads) over host memory, N = 2/4/8, against
numpy. The same contract is run on the GPU by tests/test_gpu_comm.py (RCCL at
world size 1, the one-shot IPC all-reduce at world size 1 and with two ranks
sharing one GPU). Reference: the partial combine and the groupBy shuffle of
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:500,524-525,576,732-750."""
import threading

import numpy as np
import pytest
import torch

from tensorframes_amd._native import _C

DTYPES = [torch.float32, torch.float64, torch.int32, torch.int64]
OPS = {"Sum": np.add.reduce, "Min": np.minimum.reduce, "Max": np.maximum.reduce, "Prod": np.multiply.reduce}


def _run(n, fn):
    """fn(comm, rank) on n threads; returns the per-rank results."""
    world = _C.FakeWorld(n)
    out, errs = [None] * n, []

    def body(r):
        try:
            out[r] = fn(world.comm(r), r)
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, "; ".join(str(e) for e in errs)
    return out


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", list(OPS))
def test_all_reduce(n, dtype, op):
    rng = np.random.default_rng(n)
    vals = [rng.integers(1, 5, size=(3, 5)).astype(np.float64) for _ in range(n)]

    def fn(c, r):
        t = torch.from_numpy(vals[r]).to(dtype).clone()  # the reduce is in place
        c.all_reduce(t, op)
        return t.numpy().astype(np.float64)

    got = _run(n, fn)
    want = OPS[op](np.stack(vals), axis=0)
    for g in got:
        np.testing.assert_allclose(g, want, rtol=1e-6)
    # every rank holds bitwise the same result
    assert all(np.array_equal(got[0], g) for g in got)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_all_gather_and_broadcast(n):
    def fn(c, r):
        g = c.all_gather(torch.full((2, 3), float(r)))
        b = torch.full((4,), float(r))
        c.broadcast(b, n - 1)
        c.barrier()
        return g.numpy(), b.numpy(), c.calls

    for g, b, calls in _run(n, fn):
        assert g.shape == (n, 2, 3)
        np.testing.assert_array_equal(g[:, 0, 0], np.arange(n))
        np.testing.assert_array_equal(b, np.full(4, n - 1.0))
        assert calls == 2


@pytest.mark.parametrize("n", [2, 4, 8])
def test_all_to_all_v(n):
    """Rank s sends (s + r) % 3 rows to rank r, each row tagged (s, r, i)."""
    def rows(s, r):
        return (s + r) % 3

    def fn(c, s):
        chunks = [torch.tensor([[s, r, i] for i in range(rows(s, r))], dtype=torch.int64).reshape(-1, 3)
                  for r in range(n)]
        x = torch.cat(chunks, 0)
        got = c.all_to_all_v(x, [rows(s, r) for r in range(n)], [rows(q, s) for q in range(n)])
        return got.numpy()

    for r, got in enumerate(_run(n, fn)):
        want = np.array([[s, r, i] for s in range(n) for i in range(rows(s, r))], dtype=np.int64).reshape(-1, 3)
        np.testing.assert_array_equal(got, want)


def test_mismatched_counts_raise():
    def fn(c, r):
        x = torch.zeros((2, 1))
        # rank 0 expects 5 rows from rank 1, which sends 1
        return c.all_to_all_v(x, [1, 1], [1, 5] if r == 0 else [1, 1])

    with pytest.raises(AssertionError, match="all_to_all_v"):
        _run(2, fn)

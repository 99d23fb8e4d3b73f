"""The shared-memory host communicator (csrc/comm ShmComm) at world 2, 4 and 8:
every collective of the engine's Comm contract against a plain-PyTorch
oracle, payloads larger than a slot (several rounds), zero-size tensors,
skewed all-to-all counts, and the bounded barrier (a rank that never joins
makes the others raise CollectiveError; the segment is then poisoned so the
late rank fails fast too). Reference counterpart: the driver-side combine and
shuffle of DebugRowOps.scala:500, :524-525, :576."""
import json
import os
import socket
import sys
import time
import uuid

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


def _counts(world, seed=0):
    g = torch.Generator().manual_seed(seed)
    c = torch.randint(0, 40, (world, world), generator=g)
    c[0, world - 1] = 0  # an empty pair
    c[world - 1, 0] = 3000  # a pair larger than one round
    return c


def _worker(rank, world, port, name, slot, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, REPO)
    torch.set_num_threads(1)
    import torch.distributed as td
    from tensorframes_amd._native import _C
    td.init_process_group("gloo", rank=rank, world_size=world)
    c = _C.ShmComm(name, 0, world, slot, True) if rank == 0 else None
    td.barrier()
    if rank:
        c = _C.ShmComm(name, rank, world, slot, False)
    td.barrier()
    if rank == 0:
        assert c.attached == world
        c.unlink()
    res = {}
    # all_reduce: small (every rank folds) and large (scatter-fold, several rounds)
    t = torch.arange(1000, dtype=torch.float64) * (rank + 1)
    c.all_reduce(t, "Sum")
    res["small_sum"] = bool(torch.equal(t, torch.arange(1000, dtype=torch.float64) * (world * (world + 1) // 2)))
    big = torch.arange(3 << 20, dtype=torch.float32) % 1024 + rank
    c.all_reduce(big, "Max")
    res["big_max"] = bool(torch.equal(big, torch.arange(3 << 20, dtype=torch.float32) % 1024 + (world - 1)))
    bigs = torch.full((700_001,), float(rank + 1), dtype=torch.float64)
    c.all_reduce(bigs, "Sum")
    res["big_sum"] = bool((bigs == world * (world + 1) / 2).all())
    mn = torch.tensor([rank - 5, 7 * rank, 100], dtype=torch.int64)
    c.all_reduce(mn, "Min")
    res["min"] = mn.tolist()
    pr = torch.tensor([2, rank + 1], dtype=torch.int32)
    c.all_reduce(pr, "Prod")
    res["prod"] = pr.tolist()
    z = torch.empty(0, dtype=torch.float32)
    c.all_reduce(z, "Sum")
    # all_gather (several rounds at the small slot)
    g = torch.full((50_000, 3), rank, dtype=torch.int32)
    ga = c.all_gather(g)
    res["gather"] = bool(all(torch.equal(ga[r], torch.full((50_000, 3), r, dtype=torch.int32)) for r in range(world)))
    res["gather0"] = list(c.all_gather(torch.empty((0, 2))).shape)
    # broadcast from the last rank
    b = torch.arange(300_000, dtype=torch.int64) if rank == world - 1 else torch.zeros(300_000, dtype=torch.int64)
    c.broadcast(b, world - 1)
    res["bcast"] = bool(torch.equal(b, torch.arange(300_000, dtype=torch.int64)))
    # all_to_all_v with skewed counts: row = (src, dst, i)
    cnt = _counts(world)
    send = cnt[rank].tolist()
    rows = []
    for d in range(world):
        i = torch.arange(send[d], dtype=torch.float64)
        rows.append(torch.stack([torch.full_like(i, rank), torch.full_like(i, d), i], 1))
    x = torch.cat(rows, 0)
    recv = cnt[:, rank].tolist()
    got = c.all_to_all_v(x, send, recv)
    want = torch.cat([torch.stack([torch.full((recv[s],), float(s), dtype=torch.float64),
                                   torch.full((recv[s],), float(rank), dtype=torch.float64),
                                   torch.arange(recv[s], dtype=torch.float64)], 1) for s in range(world)], 0)
    res["a2a"] = bool(torch.equal(got, want))
    # a mismatched receive count raises on every rank (none is left waiting)
    bad = list(recv)
    if rank == 0:
        bad[0] += 1
    try:
        c.all_to_all_v(x, send, bad)
        res["a2a_bad"] = "no error"
    except (_C.CollectiveError, ValueError, RuntimeError) as e:
        res["a2a_bad"] = type(e).__name__
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shm_collectives(world, tmp_path):
    name = f"/tfa_test_{uuid.uuid4().hex[:12]}"
    mp.spawn(_worker, args=(world, _free_port(), name, 256 << 10, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        o = json.load(open(tmp_path / f"r{r}.json"))
        assert o["small_sum"] and o["big_max"] and o["big_sum"], o
        assert o["min"] == [-5, 0, 100]
        import math
        assert o["prod"] == [2 ** world, math.factorial(world)]
        assert o["gather"] and o["gather0"] == [world, 0, 2]
        assert o["bcast"] and o["a2a"]
        assert o["a2a_bad"] != "no error"
    assert not os.path.exists("/dev/shm" + name)  # unlinked once attached


def _timeout_worker(rank, world, port, name, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, REPO)
    import torch.distributed as td
    from tensorframes_amd._native import _C
    td.init_process_group("gloo", rank=rank, world_size=world)
    c = _C.ShmComm(name, 0, world, 1 << 16, True) if rank == 0 else None
    td.barrier()
    if rank:
        c = _C.ShmComm(name, rank, world, 1 << 16, False)
    td.barrier()
    c.set_timeout(1.0)
    t0 = time.time()
    res = {}
    if rank == 0:
        time.sleep(3.0)  # never joins in time
    try:
        c.barrier()
        res["err"] = None
    except _C.CollectiveError as e:
        res["err"] = str(e)
    res["secs"] = time.time() - t0
    with open(os.path.join(outdir, f"t{rank}.json"), "w") as f:
        json.dump(res, f)
    td.destroy_process_group()


def test_shm_barrier_timeout(tmp_path):
    name = f"/tfa_test_{uuid.uuid4().hex[:12]}"
    mp.spawn(_timeout_worker, args=(3, _free_port(), name, str(tmp_path)), nprocs=3, join=True)
    outs = [json.load(open(tmp_path / f"t{r}.json")) for r in range(3)]
    for r in (1, 2):
        assert outs[r]["err"] is not None and outs[r]["secs"] < 2.9, outs[r]
    assert outs[1]["err"].find("timed out") >= 0 or outs[2]["err"].find("timed out") >= 0
    # the late rank finds the segment poisoned and fails at once
    # (3 s asleep, then no wait of its own: a full 1 s timeout would make it
    # >= 4 s; < 3.9 s leaves room for a loaded host)
    assert outs[0]["err"] is not None and outs[0]["secs"] < 3.9


def test_fake_world_contract_unchanged():
    from tensorframes_amd._native import _C
    w = _C.FakeWorld(1)
    c = w.comm(0)
    t = torch.ones(3)
    c.all_reduce(t, "Sum")
    assert t.tolist() == [1.0, 1.0, 1.0] and c.kind == "fake"

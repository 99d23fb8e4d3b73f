"""Device groupBy segmentation (kernels/groupby.hip) and aggregate.

CPU: the ATen oracle path of the same helpers, and size-bucketed batched
execution of non-monoid reducer graphs. GPU: radix-sort factorisation,
key hash routing, and aggregate over 10M rows / 100k integer keys against a
numpy oracle (reference: DebugRowOps.scala:547-695)."""
import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd._native import _C
from tensorframes_amd.ops import groupby as G
from tensorframes_amd.utils.logging import metrics


def _check_group_ids(keys, ids, uniq, ng):
    kn = [k.cpu().numpy() for k in keys]
    tuples = list(zip(*kn))
    want = sorted(set(tuples))
    assert ng == len(want)
    got_uniq = list(zip(*[u.cpu().numpy() for u in uniq]))
    assert got_uniq == want  # ascending (lexicographic) key order
    idn = ids.cpu().numpy()
    for i in range(0, len(tuples), max(1, len(tuples) // 500)):
        assert want[idn[i]] == tuples[i]


@pytest.mark.parametrize("dt", [torch.int32, torch.int64, torch.float32, torch.float64])
def test_group_ids_cpu(dt):
    k = torch.tensor(np.random.default_rng(0).integers(-50, 50, 1000)).to(dt)
    ids, uniq, ng = G.group_ids([k])
    _check_group_ids([k], ids, uniq, ng)


def test_group_ids_two_keys_cpu():
    rng = np.random.default_rng(1)
    a = torch.tensor(rng.integers(0, 7, 3000))
    b = torch.tensor(rng.integers(-3, 3, 3000)).to(torch.int32)
    ids, uniq, ng = G.group_ids([a, b])
    _check_group_ids([a, b], ids, uniq, ng)


def test_generic_aggregate_runs_equal_size_groups_batched():
    n = 1200
    k = np.arange(n) % 40
    x = np.random.default_rng(2).standard_normal((n, 3))
    df = tfs.from_columns({"k": k, "x": x}, num_partitions=3)
    before = metrics.snapshot().get("aggregate_batched_groups", 0)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None, 3], name="x_input")
        # not a monoid: rows are grouped, then the graph runs on each group's block
        out = tfs.aggregate(tf.identity(tf.reduce_max(xi, [0]) - tf.reduce_min(xi, [0]), name="x"), df.groupBy("k"))
        rows = sorted(out.collect(), key=lambda r: r.k)
    assert metrics.snapshot().get("aggregate_batched_groups", 0) - before == 40
    for r in rows:
        g = x[k == r.k]
        np.testing.assert_allclose(r.x, g.max(0) - g.min(0))


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.int32, torch.int64, torch.float32, torch.float64])
def test_factorize_gpu(dt):
    dev = _gpu()
    k = torch.tensor(np.random.default_rng(3).integers(-1000, 1000, 100_003)).to(dt).to(dev)
    ids, uniq, ng = G.group_ids([k])
    assert ids.is_cuda and uniq[0].is_cuda
    _check_group_ids([k], ids, uniq, ng)
    ids_c, uniq_c, ng_c = G.group_ids([k.cpu()])
    assert ng == ng_c and torch.equal(ids.cpu(), ids_c) and torch.equal(uniq[0].cpu(), uniq_c[0])


@pytest.mark.gpu
def test_factorize_two_keys_and_routing_gpu():
    dev = _gpu()
    rng = np.random.default_rng(4)
    a = torch.tensor(rng.integers(0, 100, 50_000)).to(dev)
    b = torch.tensor(rng.integers(-5, 5, 50_000), dtype=torch.int32).to(dev)
    ids, uniq, ng = G.group_ids([a, b])
    _check_group_ids([a, b], ids, uniq, ng)
    dest = _C.key_dest([a, b], 8)
    assert int(dest.min()) >= 0 and int(dest.max()) < 8
    # same key -> same destination
    d = dest.cpu().numpy()
    pairs = {}
    for x, y, r in zip(a.cpu().numpy()[:5000], b.cpu().numpy()[:5000], d[:5000]):
        assert pairs.setdefault((x, y), r) == r
    perm, counts = _C.partition_rows(dest, 8)
    assert int(counts.sum()) == 50_000
    sd = dest[perm].cpu().numpy()
    assert (np.diff(sd) >= 0).all()  # ordered by destination
    assert np.array_equal(np.bincount(d, minlength=8), counts.cpu().numpy())


@pytest.mark.gpu
def test_aggregate_10m_rows_100k_keys_gpu():
    dev = _gpu()
    n, nk = 10_000_000, 100_000
    g = torch.Generator(device=dev).manual_seed(5)
    keys = torch.randint(0, nk, (n,), device=dev, generator=g, dtype=torch.int64)
    x = torch.rand((n, 4), device=dev, generator=g, dtype=torch.float64)
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=4).cache_on_device(dev)
    before = metrics.snapshot().get("aggregate_device_groupby", 0)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None, 4], name="x_input")
        out = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k"))
        blk = out.local_blocks()
    assert metrics.snapshot().get("aggregate_device_groupby", 0) - before == 1
    (b,) = blk.values()
    kk, xx = b.columns["k"].cpu().numpy(), b.columns["x"].cpu().numpy()
    kn, xn = keys.cpu().numpy(), x.cpu().numpy()
    want_k = np.unique(kn)
    assert np.array_equal(kk, want_k)
    want = np.zeros((nk, 4))
    np.add.at(want, kn, xn)
    np.testing.assert_allclose(xx, want[want_k], rtol=1e-10, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("op,fn", [("Sum", "unsorted_segment_sum"), ("Max", "unsorted_segment_max"),
                                   ("Min", "unsorted_segment_min")])
@pytest.mark.parametrize("inner", [1, 3, 64, 100])
def test_unsorted_segment_many_segments_gpu(op, fn, inner):
    """More segments than the LDS-private kernel holds: rows are ordered by
    segment with a radix sort and reduced per segment (deterministic)."""
    dev = _gpu()
    if not hasattr(tf, fn):
        pytest.skip(f"DSL has no {fn}")
    nseg = 5000
    rng = np.random.default_rng(6)
    x = rng.standard_normal((40_000, inner))
    ids = rng.integers(-3, nseg + 3, 40_000).astype(np.int32)  # out-of-range ids drop out
    g = tf.Graph()
    with g.as_default():
        xp = tf.placeholder(tf.double, [None, inner], name="x")
        ip = tf.placeholder(tf.int32, [None], name="ids")
        getattr(tf, fn)(xp, ip, nseg, name="y")
    from tensorframes_amd import engine
    prog = engine.program(g.serialize(), ["y"], ["x", "ids"])
    want = engine.run_program(prog, [torch.from_numpy(x), torch.from_numpy(ids)], torch.device("cpu"))[0]
    got = engine.run_program(prog, [torch.from_numpy(x), torch.from_numpy(ids)], dev)[0].cpu()
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)
    again = engine.run_program(prog, [torch.from_numpy(x), torch.from_numpy(ids)], dev)[0].cpu()
    assert torch.equal(got, again)  # deterministic


def _float_keys_with_specials(n, dt, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(-20, 20, n).astype(np.float64) / 4
    k[rng.random(n) < 0.05] = np.nan
    k[rng.random(n) < 0.05] = -0.0
    k[rng.random(n) < 0.02] = np.inf
    k[rng.random(n) < 0.02] = -np.inf
    nan2 = np.frombuffer(np.uint64(0xfff8000000000001).tobytes(), np.float64)[0]  # another NaN payload
    k[rng.random(n) < 0.02] = nan2
    return torch.tensor(k).to(dt)


def _check_special_groups(k, ids, uniq, ng):
    kn = k.cpu().double().numpy()
    u = uniq[0].cpu().double().numpy()
    want = np.unique(np.where(kn == 0, 0.0, kn))  # numpy: NaNs equal, one group last
    assert ng == len(want), (ng, want)
    np.testing.assert_array_equal(u, want)
    assert not np.signbit(u[u == 0]).any()  # the zero group is +0.0
    idn = ids.cpu().numpy()
    canon = np.where(np.isnan(kn), np.inf * 2, kn)  # compare NaN as one value
    wantc = np.where(np.isnan(want), np.inf * 2, want)
    assert np.array_equal(wantc[idn], np.where(canon == 0, 0.0, canon))


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_group_ids_nan_and_signed_zero_keys_cpu(dt):
    k = _float_keys_with_specials(5000, dt, 7)
    ids, uniq, ng = G.group_ids([k])
    _check_special_groups(k, ids, uniq, ng)


def test_key_hash_routes_equal_float_keys_together():
    from tensorframes_amd.core import _key_hash
    nan2 = np.frombuffer(np.uint64(0xfff8000000000001).tobytes(), np.float64)[0]
    a = np.array([np.nan, nan2, 0.0, -0.0])
    h = _key_hash([a])
    assert h[0] == h[1] and h[2] == h[3]


def test_aggregate_nan_keys_form_one_group():
    k = np.array([1.0, np.nan, -0.0, 0.0, np.nan, 1.0])
    x = np.arange(6, dtype=np.float64)
    df = tfs.from_columns({"k": k, "x": x}, num_partitions=2)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        rows = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k")).collect()
    got = {("nan" if np.isnan(r.k) else float(r.k)): float(r.x) for r in rows}
    assert got == {0.0: 5.0, 1.0: 5.0, "nan": 5.0}


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_factorize_nan_and_signed_zero_keys_gpu(dt):
    dev = _gpu()
    k = _float_keys_with_specials(200_001, dt, 8)
    ids, uniq, ng = G.group_ids([k.to(dev)])
    _check_special_groups(k, ids, uniq, ng)
    ids_c, uniq_c, ng_c = G.group_ids([k])
    assert ng == ng_c and torch.equal(ids.cpu(), ids_c)
    assert torch.equal(uniq[0].cpu().isnan(), uniq_c[0].isnan())
    dest = _C.key_dest([k.to(dev)], 8).cpu().numpy()
    kn = k.double().numpy()
    assert len(set(dest[np.isnan(kn)])) == 1 and len(set(dest[kn == 0])) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["dense", "narrow_sort", "wide", "single", "one_tile"])
@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_factorize_int_paths_gpu(kind, dt):
    """The dense (direct-address), narrow radix-sort and full-width radix-sort
    factorisations agree with the host oracle; sizes straddle the 4096-key
    sort tile and the 2048-element scan tile."""
    dev = _gpu()
    rng = np.random.default_rng(9)
    n = {"dense": 3_000_017, "narrow_sort": 1_000_003, "wide": 777_777, "single": 1, "one_tile": 4095}[kind]
    if kind == "dense":
        k = rng.integers(-50_000, 50_000, n)
    elif kind == "narrow_sort":  # range >> rows: sorted on the bits of key - min
        k = rng.integers(0, 1 << 30, n) * (1 if dt == torch.int64 else 1) - (1 << 29)
    elif kind == "wide":
        if dt == torch.int32:
            k = rng.integers(-(1 << 31), (1 << 31) - 1, n)
        else:
            k = rng.integers(-(1 << 62), 1 << 62, n)
    else:
        k = rng.integers(-3, 1 << 20, n)
    kt = torch.tensor(k).to(dt)
    ids, uniq, ng = G.group_ids([kt.to(dev)])
    want_u, want_inv = np.unique(kt.numpy(), return_inverse=True)
    assert ng == len(want_u)
    np.testing.assert_array_equal(uniq[0].cpu().numpy(), want_u)
    np.testing.assert_array_equal(ids.cpu().numpy(), want_inv.reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 3, 8, 256])
def test_partition_rows_is_stable_gpu(world):
    dev = _gpu()
    n = 300_001
    dest = torch.tensor(np.random.default_rng(10).integers(0, world, n)).to(dev)
    perm, counts = _C.partition_rows(dest, world)
    p = perm.cpu().numpy()
    want = np.argsort(dest.cpu().numpy(), kind="stable")
    np.testing.assert_array_equal(p, want)
    np.testing.assert_array_equal(counts.cpu().numpy(), np.bincount(dest.cpu().numpy(), minlength=world))


def _range_graph(width):
    xi = tf.placeholder(tf.double, [None, width], name="x_input")
    # not a monoid: per-key range (max - min) of every column
    return tf.identity(tf.reduce_max(xi, [0]) - tf.reduce_min(xi, [0]), name="x")


@pytest.mark.gpu
def test_generic_aggregate_device_matches_numpy_gpu():
    dev = _gpu()
    rng = np.random.default_rng(11)
    n = 200_003
    k = rng.integers(-500, 1500, n)
    k[:7] = 99_999  # one big group, and sizes that occur once
    x = rng.standard_normal((n, 2))
    df = tfs.from_columns({"k": torch.tensor(k).to(dev), "x": torch.tensor(x).to(dev)},
                          num_partitions=3).cache_on_device(dev)
    before = metrics.snapshot().get("aggregate_device_generic", 0)
    with tf.Graph().as_default():
        blk = tfs.aggregate(_range_graph(2), df.groupBy("k")).local_blocks()
    assert metrics.snapshot().get("aggregate_device_generic", 0) - before == 1
    (b,) = blk.values()
    kk, xx = b.columns["k"].cpu().numpy(), b.columns["x"].cpu().numpy()
    want_k, inv = np.unique(k, return_inverse=True)
    assert np.array_equal(kk, want_k)
    mx = np.full((len(want_k), 2), -np.inf)
    mn = np.full((len(want_k), 2), np.inf)
    np.maximum.at(mx, inv.reshape(-1), x)
    np.minimum.at(mn, inv.reshape(-1), x)
    np.testing.assert_array_equal(xx, mx - mn)


@pytest.mark.gpu
def test_generic_aggregate_10m_rows_100k_keys_gpu():
    """a non-monoid aggregate over 10M device-cached rows /
    100k keys in < 50 ms (round 2: host pandas/np.unique + per-group loop)."""
    import time
    dev = _gpu()
    n, nk = 10_000_000, 100_000
    g = torch.Generator(device=dev).manual_seed(12)
    keys = torch.randint(0, nk, (n,), device=dev, generator=g, dtype=torch.int64)
    x = torch.rand((n, 4), device=dev, generator=g, dtype=torch.float64)
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=4).cache_on_device(dev)
    with tf.Graph().as_default():
        gr = _range_graph(4)
        tfs.aggregate(gr, df.groupBy("k")).local_blocks()  # lifts + plans once per group size
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blk = tfs.aggregate(gr, df.groupBy("k")).local_blocks()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    (b,) = blk.values()
    assert b.nrows == nk
    print(f"generic aggregate 10M rows / 100k keys: {dt * 1e3:.1f} ms")
    kn = keys.cpu().numpy()
    xn = x.cpu().numpy()
    sel = np.nonzero(kn == 12345)[0]
    np.testing.assert_array_equal(b.columns["x"][12345].cpu().numpy(), xn[sel].max(0) - xn[sel].min(0))
    assert dt < 0.05, dt


@pytest.mark.gpu
def test_pack_unpack_records_roundtrip_gpu():
    """The keyed shuffle's single-payload records: every column of a row in
    one word-aligned record (pack_rows), restored by unpack_rows."""
    dev = _gpu()
    rng = np.random.default_rng(13)
    n = 10_007
    cols = [torch.tensor(rng.integers(-9, 9, n)).to(dev),
            torch.tensor(rng.standard_normal((n, 4))).to(dev),
            torch.tensor(rng.integers(0, 5, n), dtype=torch.int32).to(dev),
            torch.tensor(rng.integers(0, 255, (n, 3)), dtype=torch.uint8).to(dev)]
    perm = torch.tensor(rng.permutation(n)).to(dev)
    rec, offs = _C.pack_rows(cols, perm)
    assert rec.shape == (n, 8 + 32 + 4 + 4) and list(offs) == [0, 8, 40, 44]
    outs = [torch.empty_like(c) for c in cols]
    _C.unpack_rows(rec, outs)
    for c, o in zip(cols, outs):
        assert torch.equal(o, c[perm])
    # all-float columns take the word path, a lone uint8 column the byte path
    rec2, _ = _C.pack_rows([cols[3]])
    back = torch.empty_like(cols[3])
    _C.unpack_rows(rec2, [back])
    assert rec2.shape == (n, 4) and torch.equal(back, cols[3])


def test_pinned_pool_cap_is_bounded_by_host_ram():
    st = _C.pinned_pool_stats()
    import os
    ram = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    assert 0 < st["limit"] <= min(64 << 30, ram // local // 2) or os.environ.get("TFA_PINNED_POOL_MB")
    assert st["live"] >= 0 and st["peak"] >= st["live"]


def test_pinned_pool_cap_scales_with_local_ranks():
    import os
    import subprocess
    import sys
    code = "from tensorframes_amd._native import _C; print(_C.pinned_pool_stats()['limit'])"

    def limit(local):
        env = {k: v for k, v in os.environ.items() if k != "TFA_PINNED_POOL_MB"}
        env["LOCAL_WORLD_SIZE"] = str(local)
        return int(subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                                  check=True).stdout.strip())
    ram = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    assert limit(8) == min(64 << 30, ram // 8 // 2)
    assert limit(1) == min(64 << 30, ram // 2)

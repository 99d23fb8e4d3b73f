"""groupBy on string / binary keys without Python objects per row: the keys
are Arrow-layout StringColumns (offsets + bytes) packed into big-endian words
+ length (`_C.string_words`) and grouped by the numeric kernels, exactly and in
lexicographic order. Reference: src/main/python/tensorframes/core_test.py:118-127
(groupBy a string key) and DebugRowOps.scala:547-592 (aggregate)."""
import json
import os
import socket
import sys

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd._native import _C
from tensorframes_amd.frame.block import StringColumn
from tensorframes_amd.ops import groupby as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_string_words_order_and_roundtrip():
    vals = ["", "a", "a\x00", "ab", "abcdefgh", "abcdefghi", "b", "zz", "é", "日本語のキー", "abcdefgh" * 3]
    col = StringColumn.from_values(vals)
    w = G.string_width([col])
    assert w == 3
    words = G.string_key_words(col, w, torch.device("cpu"))
    assert len(words) == w + 1
    # signed order of (words..., length) == lexicographic order of the UTF-8 bytes
    keyt = list(zip(*[c.tolist() for c in words]))
    assert sorted(range(len(vals)), key=lambda i: keyt[i]) == sorted(range(len(vals)),
                                                                      key=lambda i: vals[i].encode())
    back = G.words_to_strings(words)
    assert back.values == vals


def test_string_column_layouts():
    arr = np.array(["x1", "yy22", "", "zzz333"])
    c = StringColumn.from_numpy(arr)
    assert c.values == arr.tolist() and len(c) == 4
    assert c.slice(1, 3).values == ["yy22", ""]
    assert c.take([3, 0, 3]).values == ["zzz333", "x1", "zzz333"]
    from tensorframes_amd.frame.block import concat_columns
    assert concat_columns([c.slice(0, 2), c.slice(2, 4)]).values == arr.tolist()


def _agg(df, key, dtype=np.float64):
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        return tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy(key)).collect()


def test_core_test_groupby_parity():
    """core_test.py:118-127: key = str(x % 2) -> [Row(key='0', x=2.0), Row(key='1', x=4.0)]."""
    df = tfs.create_dataframe([tfs.Row(x=float(x), key=str(x % 2)) for x in range(4)])
    rows = _agg(df, "key")
    assert rows == [tfs.Row(key="0", x=2.0), tfs.Row(key="1", x=4.0)]


@pytest.mark.parametrize("nparts", [1, 3])
def test_string_key_aggregate_matches_pandas(nparts):
    rng = np.random.default_rng(0)
    pool = np.array([f"key{i:04d}" + "x" * (i % 13) for i in range(300)] + ["", "é", "日本"])
    keys = pool[rng.integers(0, len(pool), 20000)]
    x = rng.standard_normal(20000)
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=nparts)
    assert isinstance(df.local_blocks()[0].columns["k"], StringColumn)
    rows = _agg(df, "k")
    want = pd.Series(x).groupby(keys).sum()
    got_keys = [r.k for r in rows]
    assert got_keys == sorted(got_keys, key=lambda s: s.encode())  # lexicographic group order
    assert got_keys == sorted(want.index.tolist(), key=lambda s: s.encode())
    np.testing.assert_allclose([r.x for r in rows], want[got_keys].to_numpy(), rtol=1e-10)


def test_string_and_int_keys_together():
    rng = np.random.default_rng(1)
    s = np.array(["a", "bb", "ccc"])[rng.integers(0, 3, 5000)]
    i = rng.integers(0, 4, 5000).astype(np.int64)
    x = rng.standard_normal(5000)
    df = tfs.from_columns({"s": s, "i": i, "x": x}, num_partitions=2)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        rows = tfs.aggregate(tf.reduce_max(xi, [0], name="x"), df.groupBy("s", "i")).collect()
    want = pd.DataFrame({"s": s, "i": i, "x": x}).groupby(["s", "i"])["x"].max()
    assert [(r.s, r.i) for r in rows] == list(want.index)
    np.testing.assert_allclose([r.x for r in rows], want.to_numpy())


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TFA_DEVICE="cpu", OMP_NUM_THREADS="1")
    sys.path.insert(0, REPO)
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.parallel import dist
    from tensorframes_amd.utils.logging import metrics
    assert dist.init(backend="gloo")
    rng = np.random.default_rng(7)
    keys = np.array([f"user-{i % 97:03d}" * (1 + i % 3) for i in range(6000)])
    x = rng.standard_normal(6000)
    df = tfs.from_columns({"k": keys, "x": x}, num_partitions=world + 1)
    metrics.reset()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        rows = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k")).collect()
    m = metrics.snapshot()
    res = {"keys": [r.k for r in rows], "x": [r.x for r in rows],
           "pickles": sum(m.get(f"collective_{k}", 0) for k in ("all_to_all_objects", "all_gather_object"))}
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.shutdown()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_string_keys_shuffle_without_pickling(world, tmp_path):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    keys = np.array([f"user-{i % 97:03d}" * (1 + i % 3) for i in range(6000)])
    x = np.random.default_rng(7).standard_normal(6000)
    want = pd.Series(x).groupby(keys).sum()
    for r in range(world):
        res = json.load(open(tmp_path / f"r{r}.json"))
        assert res["pickles"] == 0  # keys travelled as packed int64 words, not pickled str
        got = dict(zip(res["keys"], res["x"]))
        assert set(got) == set(want.index)
        np.testing.assert_allclose([got[k] for k in want.index], want.to_numpy(), rtol=1e-9)


def test_long_keys_bounded_width_exact_order():
    """Keys longer than 8 bytes group on (word 0, tag = 9 + 62-bit hash): 2
    words per row however long the longest key (one 4 KB key here), exact
    against pandas, in lexicographic order even among long keys that share
    their first 8 bytes (those sort by hash until re-ordered)."""
    from tensorframes_amd.utils.logging import metrics
    rng = np.random.default_rng(3)
    pool = ["shared__" + "z" * int(n) + str(i) for i, n in enumerate(rng.integers(0, 30, 60))]
    pool += ["shared__", "shared_", "shared__a", "s", "", "x" * 4096, "x" * 4095 + "y", "é" * 9]
    keys = np.array(pool, dtype=object)[rng.integers(0, len(pool), 30000)]
    x = rng.standard_normal(30000)
    df = tfs.from_columns({"k": keys.astype(str), "x": x}, num_partitions=3)
    metrics.reset()
    rows = _agg(df, "k")
    assert metrics.snapshot().get("aggregate_string_key_words") == 2  # word 0 + tag
    want = pd.Series(x).groupby(keys.astype(str)).sum()
    got_keys = [r.k for r in rows]
    assert got_keys == sorted(want.index.tolist(), key=lambda s: s.encode())
    np.testing.assert_allclose([r.x for r in rows], want[got_keys].to_numpy(), rtol=1e-10)


def test_long_string_and_int_keys_order():
    rng = np.random.default_rng(4)
    s = np.array(["prefix__" + "q" * int(n) for n in range(12)] + ["prefix__b" * 3])[rng.integers(0, 13, 8000)]
    i = rng.integers(0, 3, 8000).astype(np.int64)
    x = rng.standard_normal(8000)
    df = tfs.from_columns({"s": s, "i": i, "x": x}, num_partitions=2)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        rows = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("s", "i")).collect()
    want = pd.DataFrame({"s": s, "i": i, "x": x}).groupby(["s", "i"])["x"].sum()
    assert [(r.s, r.i) for r in rows] == sorted(want.index, key=lambda t: (t[0].encode(), t[1]))
    got = {(r.s, r.i): r.x for r in rows}
    np.testing.assert_allclose([got[t] for t in want.index], want.to_numpy(), rtol=1e-10)


def test_hash_collision_is_detected_and_falls_back(monkeypatch):
    """A (forced) hash collision: every long key gets the same hash. The
    per-group verification catches it and the aggregation reruns on exact
    words; the result is still exact."""
    from tensorframes_amd.utils.logging import metrics
    real = G.string_key_hashed

    def colliding(col, dev):
        w0, t = real(col, dev)
        return [w0, torch.where(t >= G.HASH_TAG_MIN, torch.full_like(t, G.HASH_TAG_MIN), t)]
    monkeypatch.setattr(G, "string_key_hashed", colliding)
    keys = np.array(["collide_" + "a" * 20, "collide_" + "b" * 20, "short"])[np.arange(300) % 3]
    x = np.arange(300, dtype=np.float64)
    df = tfs.from_columns({"k": keys, "x": x})
    metrics.reset()
    rows = _agg(df, "k")
    assert metrics.snapshot().get("aggregate_string_key_collisions") == 1
    want = pd.Series(x).groupby(keys).sum()
    assert [r.k for r in rows] == list(want.index)
    np.testing.assert_allclose([r.x for r in rows], want.to_numpy())


def test_group_keys_verification_direct():
    col = StringColumn.from_values(["same_pre_" + "1" * 10, "same_pre_" + "2" * 10])
    w0, t = G.string_key_hashed(col, torch.device("cpu"))
    with pytest.raises(G.StringKeyCollision):
        G.group_keys([w0, torch.full_like(t, G.HASH_TAG_MIN)], {0: col})
    ids, uniq, ng, ustr = G.group_keys([w0, t], {0: col})
    assert ng == 2 and ustr[0].values == sorted(col.values)

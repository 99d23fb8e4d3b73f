"""String-key groupBy on the GPU: 10M rows / 100k string keys (Arrow layout,
bytes in HBM), monoid graph — the keys are packed into words by
`_C.string_words` and grouped by the numeric radix kernels (no Python object
per row, no host factorisation). Reference: core_test.py:118-127 and
DebugRowOps.scala:547-592."""
import time

import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.frame.block import StringColumn
from tensorframes_amd.utils.logging import metrics

pytestmark = pytest.mark.gpu


def _keys(ids: np.ndarray) -> StringColumn:
    """'k' + 6 decimal digits per id, built as bytes (vectorised)."""
    digits = (ids[:, None] // (10 ** np.arange(5, -1, -1))[None, :]) % 10 + ord("0")
    raw = np.concatenate([np.full((len(ids), 1), ord("k")), digits], 1).astype(np.uint8)
    offs = np.arange(len(ids) + 1, dtype=np.int64) * 7
    return StringColumn(torch.from_numpy(offs), torch.from_numpy(raw.reshape(-1)))


def test_string_key_aggregate_10m_rows_100k_keys_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    n, nk = 10_000_000, 100_000
    rng = np.random.default_rng(3)
    ids = rng.integers(0, nk, n)
    x = rng.standard_normal((n, 4))
    df = tfs.from_columns({"k": _keys(ids), "x": x}, num_partitions=4).cache_on_device(dev)
    assert df.local_blocks()[0].columns["k"].is_cuda
    times = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.double, [None, 4], name="x_input")
            out = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k"))
            (b,) = out.local_blocks().values()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    print(f"string-key aggregate 10M rows / 100k keys: {min(times) * 1e3:.1f} ms (runs {[round(t * 1e3, 1) for t in times]})")
    assert metrics.snapshot().get("aggregate_device_groupby", 0) >= 1
    keys = b.columns["k"].values
    want_ids = np.unique(ids)
    assert keys == [f"k{i:06d}" for i in want_ids]
    want = np.zeros((nk, 4))
    np.add.at(want, ids, x)
    np.testing.assert_allclose(b.columns["x"].cpu().numpy(), want[want_ids], rtol=1e-9, atol=1e-9)
    assert min(times) < 0.05, times


def test_string_keys_bounded_width_with_one_4kb_key_gpu():
    """The same 10M rows / 100k 7-byte keys plus ONE 4 KB key: the key width
    stays 2 words per row (word 0, tag = length or 9 + 62-bit hash;
    ops/groupby.py) instead of 513, and the grouping stays exact (per-group
    byte verification)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda", 0)
    n, nk = 10_000_000, 100_000
    rng = np.random.default_rng(4)
    ids = rng.integers(0, nk, n)
    x = rng.standard_normal((n, 4))
    short = _keys(ids[1:])
    big = np.full(4096, ord("L"), dtype=np.uint8)
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.tensor([4096]), short.offsets[1:] + 4096])
    col = StringColumn(offs, torch.cat([torch.from_numpy(big), short.data]))
    df = tfs.from_columns({"k": col, "x": x}, num_partitions=4).cache_on_device(dev)
    times = []
    for _ in range(4):
        metrics.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.double, [None, 4], name="x_input")
            out = tfs.aggregate(tf.reduce_sum(xi, [0], name="x"), df.groupBy("k"))
            (b,) = out.local_blocks().values()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    print(f"string-key aggregate 10M rows / 100k keys + one 4 KB key: {min(times) * 1e3:.1f} ms "
          f"(runs {[round(t * 1e3, 1) for t in times]})")
    assert metrics.snapshot().get("aggregate_string_key_words") == 2
    keys = b.columns["k"].values
    sids = np.unique(ids[1:])
    assert keys == ["L" * 4096] + [f"k{i:06d}" for i in sids]  # b"L" < b"k"
    want = np.zeros((nk, 4))
    np.add.at(want, ids[1:], x[1:])
    got = b.columns["x"].cpu().numpy()
    np.testing.assert_allclose(got[1:], want[sids], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(got[0], x[0])
    assert min(times) < 0.05, times

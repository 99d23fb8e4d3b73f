"""map_rows fast paths: a dense block runs as ONE lifted
program with no per-row Python work, so map_rows costs about what map_blocks
costs on the same work; on the GPU a lifted host block takes the same
pipelined H2D/compute/D2H path as map_blocks (chosen by block size, not cell
size). Reference: src/main/scala/org/tensorframes/impl/DebugRowOps.scala:396-477,819-857."""
import time

import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.utils.logging import metrics


def _best(fn, n=3):
    best = float("inf")
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


def test_map_rows_scalar_rows_close_to_map_blocks_cpu():
    x = np.arange(1_000_000, dtype=np.float64)
    df = tfs.from_columns({"x": x}, num_partitions=1).cache()
    df.local_blocks()

    def blocks():
        with tf.Graph().as_default():
            z = tf.add(tf.placeholder(tf.double, [None], name="x"), 3.0, name="z")
            return tfs.map_blocks(z, df).local_blocks()

    def rows():
        with tf.Graph().as_default():
            z = tf.add(tf.placeholder(tf.double, [], name="x"), 3.0, name="z")
            return tfs.map_rows(z, df).local_blocks()
    tfs.set_config(device="cpu")
    try:
        np.testing.assert_array_equal(rows()[0].columns["z"].numpy(), x + 3.0)
        tb, tr = _best(blocks), _best(rows)
    finally:
        tfs.set_config(device="auto")
    assert tr <= 2.0 * tb + 0.01, (tr, tb)  # (10 ms of slack for a loaded host)


def test_row_matmul_lifts_to_one_fused_gemm():
    """expand_dims -> MatMul -> squeeze -> relu per row becomes one
    [B,512]x[512,512] GEMM with the ReLU fused (views looked through)."""
    from tensorframes_amd.core import _LIFT_CACHE
    rng = np.random.default_rng(0)
    x = rng.standard_normal((300, 64)).astype(np.float32)
    w = rng.standard_normal((64, 32)).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=2)
    _LIFT_CACHE.clear()
    with tf.Graph().as_default():
        y = tf.nn.relu(tf.squeeze(tf.matmul(tf.expand_dims(tfs.row(df, "x"), 0), tf.constant(w)), [0]), name="y")
        got = tfs.map_rows(y, df).to_numpy("y")
    np.testing.assert_allclose(got, np.maximum(x.astype(np.float64) @ w, 0), rtol=1e-5, atol=1e-4)
    progs = [p for _, p in _LIFT_CACHE.values() if p is not None]
    assert len(progs) == 1
    plan = progs[0].describe([torch.zeros(10, 64)])
    assert "GEMM MatMul" in plan and "+relu" in plan and "1 fused epilogues" in plan


@pytest.mark.gpu
def test_row_matmul_map_rows_matches_map_blocks_throughput_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from tensorframes_amd._native import _C
    rows, dim = 1_000_000, 512
    host = _C.empty_pinned([rows, dim], torch.float32)
    host.copy_(torch.randn((rows, dim), device="cuda"))
    w = (torch.randn((dim, dim)) / dim ** 0.5).numpy()
    df = tfs.from_columns({"x": host}, num_partitions=2)

    def blocks():
        with tf.Graph().as_default():
            y = tf.nn.relu(tf.matmul(tfs.block(df, "x"), tf.constant(w)), name="y")
            return tfs.map_blocks(y, df, trim=True).local_blocks()

    def rows_():
        with tf.Graph().as_default():
            xr = tfs.row(df, "x")
            y = tf.nn.relu(tf.squeeze(tf.matmul(tf.expand_dims(xr, 0), tf.constant(w)), [0]), name="y")
            return tfs.map_rows(y, df).local_blocks()
    before = metrics.snapshot().get("map_rows_pipelined_rows", 0)
    rb, rr = blocks(), rows_()
    assert metrics.snapshot().get("map_rows_pipelined_rows", 0) - before == rows
    for p in rb:
        assert not rr[p].columns["y"].is_cuda
        torch.testing.assert_close(rr[p].columns["y"], rb[p].columns["y"], rtol=1e-5, atol=1e-5)
    tb, tr = _best(blocks), _best(rows_)
    print(f"map_blocks {rows / tb / 1e6:.2f} M rows/s, map_rows {rows / tr / 1e6:.2f} M rows/s")
    assert tr <= tb / 0.85, (tr, tb)

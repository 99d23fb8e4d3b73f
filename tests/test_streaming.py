"""Streaming actions over derived frames: partitions reach a derived
operator in bounded groups (Config.stream_group_bytes, at most 16 partitions),
so a pipelined engine call can span several partitions while memory stays
bounded; results are the same as per-partition evaluation."""
import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf
from tensorframes_amd.frame.block import Block
from tensorframes_amd.frame.dataframe import DataFrame, _Derived
from tensorframes_amd.frame.types import StructType


def _frame(nparts, rows=1000):
    schema = StructType([tfs.tensor_field("x", tf.float32, [4])])

    def make(p):
        return Block(rows, {"x": torch.full((rows, 4), float(p))})
    return tfs.generate(schema, nparts, make)


def test_derived_iteration_groups_partitions_by_bytes():
    base = _frame(10)  # 16 KB per partition
    calls = []

    def fn(blocks):
        calls.append(sorted(blocks))
        return {p: Block(b.nrows, {"x": b.columns["x"] + 1}) for p, b in blocks.items()}
    old = tfs.config.stream_group_bytes
    try:
        tfs.set_config(stream_group_bytes=40_000)
        df = DataFrame(base.schema, _Derived(base, fn), base.num_partitions)
        got = [(p, float(b.columns["x"][0, 0])) for p, b in df._iter_blocks()]
    finally:
        tfs.set_config(stream_group_bytes=old)
    assert got == [(p, p + 1.0) for p in range(10)]
    assert calls == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9]]


def test_group_partition_cap_and_map_blocks_results():
    base = _frame(40, rows=10)
    with tf.Graph().as_default():
        x = tfs.block(base, "x")
        y = tf.add(x, 3.0, name="y")
        df = tfs.map_blocks(y, base)
    assert df.count() == 400
    vals = np.concatenate([b.columns["y"].numpy() for _, b in df._iter_blocks()])
    assert vals.shape == (400, 4)
    np.testing.assert_allclose(vals[::10, 0], np.arange(40) + 3.0)


@pytest.mark.gpu
def test_streaming_groups_run_one_continuous_pipeline_gpu():
    """Host-resident partitions streamed in several groups: every group's
    chunk pipeline is enqueued before the previous one is waited for (the ring
    and slot rotation carry over, no drain between groups); results equal
    the per-row reference."""
    import pytest
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from tensorframes_amd.utils.logging import metrics
    rows, nparts = 20000, 9
    schema = StructType([tfs.tensor_field("x", tf.float32, [64])])

    def make(p):
        return Block(rows, {"x": torch.arange(rows * 64, dtype=torch.float32).reshape(rows, 64) % 97 + p})
    base = tfs.generate(schema, nparts, make)
    w = (np.arange(64 * 32, dtype=np.float32).reshape(64, 32) % 7 - 3) / 8
    old = (tfs.config.stream_group_bytes, tfs.config.min_chunked_rows, tfs.config.chunk_bytes)
    try:
        # 3 partitions per group, 4 chunks per partition
        tfs.set_config(stream_group_bytes=3 * rows * 64 * 4, min_chunked_rows=1000, chunk_bytes=rows * 64)
        with tf.Graph().as_default():
            x = tfs.block(base, "x")
            y = tf.nn.relu(tf.matmul(x, tf.constant(w)), name="y")
            df = tfs.map_blocks(y, base, trim=True)
        before = metrics.snapshot().get("pipelines_deferred", 0)
        got = [(p, b.columns["y"].numpy().copy()) for p, b in df._iter_blocks()]
        assert metrics.snapshot().get("pipelines_deferred", 0) - before == 3
    finally:
        tfs.set_config(stream_group_bytes=old[0], min_chunked_rows=old[1], chunk_bytes=old[2])
    assert [p for p, _ in got] == list(range(nparts))
    for p, y in got:
        xin = make(p).columns["x"].double().numpy()
        np.testing.assert_allclose(y, np.maximum(xin @ w.astype(np.float64), 0), rtol=1e-5, atol=1e-3)

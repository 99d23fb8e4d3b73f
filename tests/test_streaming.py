"""Streaming actions over derived frames: partitions reach a derived
operator in bounded groups (Config.stream_group_bytes, at most 16 partitions),
so a pipelined engine call can span several partitions while memory stays
bounded; results are the same as per-partition evaluation."""
import numpy as np
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

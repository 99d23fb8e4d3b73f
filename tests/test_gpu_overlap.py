"""Overlap of independent GPU work (round 6): large device-resident
map_blocks partitions run two at a time on two streams, and the host chunk
pipeline alternates chunks between two compute streams. Either way every
result must equal the one-stream run bit for bit, with the outputs ordered on
the caller's stream when they come back."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import tf  # noqa: E402
from tensorframes_amd.frame.block import Block  # noqa: E402
from tensorframes_amd.utils.logging import metrics  # noqa: E402

DEV = torch.device("cuda", 0)


def _graph(w):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 256], name="x")
        y = tf.nn.relu(tf.matmul(x, tf.constant(w)))
        tf.reduce_sum(tf.square(y), [1], name="z")
    return g


def test_large_device_partitions_two_streams_equal_serial():
    rng = np.random.default_rng(0)
    w = rng.standard_normal((256, 256)).astype(np.float32) * 0.1
    schema = tfs.StructType([tfs.tensor_field("x", tf.float32, [256])])
    parts = [torch.randn((20000 + 1000 * p, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(p))
             for p in range(5)]
    df = tfs.generate(schema, len(parts), lambda p: Block(parts[p].shape[0], {"x": parts[p]}))
    g = _graph(w)
    res = {}
    try:
        for on in (False, True):
            tfs.set_config(concurrent_large_partitions=on, concurrent_large_bytes=1 << 20)
            metrics.reset()
            with g.as_default():
                out = tfs.map_blocks(g.get_tensor_by_name("z:0"), df, trim=True).local_blocks()
            res[on] = [out[p].columns["z"].cpu().numpy() for p in range(len(parts))]
            assert (metrics.snapshot().get("concurrent_partition_runs", 0) == len(parts)) == on
    finally:
        tfs.set_config(concurrent_large_partitions=True, concurrent_large_bytes=64 << 20)
    for a, b in zip(res[False], res[True]):
        assert np.array_equal(a, b)


def test_host_pipeline_two_compute_streams_equal_reference():
    """Host-resident rows stream through the chunk pipeline (chunks alternate
    between the two compute streams); the result equals torch on the host."""
    rng = np.random.default_rng(1)
    w = rng.standard_normal((256, 256)).astype(np.float32) * 0.1
    x = rng.standard_normal((300000, 256)).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=2)
    from tensorframes_amd.config import config
    old = config.chunk_bytes
    tfs.set_config(chunk_bytes=8 << 20)
    try:
        g = _graph(w)
        with g.as_default():
            blocks = tfs.map_blocks(g.get_tensor_by_name("z:0"), df, trim=True).local_blocks()
            z = np.concatenate([blocks[p].columns["z"].cpu().numpy() for p in sorted(blocks)])
    finally:
        tfs.set_config(chunk_bytes=old)
    want = (np.maximum(x.astype(np.float64) @ w.astype(np.float64), 0) ** 2).sum(1)
    assert np.allclose(z, want, rtol=1e-4, atol=1e-3)

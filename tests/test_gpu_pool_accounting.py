"""Every device temporary of the flagship workloads comes from the engine's
stream-ordered pool (csrc/runtime/device_pool.cpp): the headline map_blocks
MatMul+ReLU over a host frame (chunk pipeline) and a device-cached one, the
K-Means demo on a device-cached frame (HIP-graph replays, reduce merge) and
Inception-v3 scoring. `fallbacks` counts pool requests that ended in
at::empty (pool disabled or out of memory); allocations made while a HIP graph
captures belong to that graph and are counted apart (`capture_allocs`)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.models import cnn, kmeans  # noqa: E402


def _headline(rows, device_cached):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((rows, 512), dtype=np.float32)
    w = (rng.standard_normal((512, 512)) / 22.6).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=4)
    if device_cached:
        df = df.cache_on_device()
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.float32, [None, 512], name="x")
        y = tf.nn.relu(tf.matmul(xi, tf.constant(w)), name="y")
        out = tfs.map_blocks(y, df)
    got = out.to_numpy("y")
    want = np.maximum(x.astype(np.float64) @ w.astype(np.float64), 0.0)
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)


def test_flagship_workloads_allocate_only_from_the_pool():
    s0 = _C.device_pool_stats()
    _headline(60000, device_cached=False)
    _headline(60000, device_cached=True)

    rng = np.random.default_rng(5)
    pts = rng.uniform(0, 1, (20000, 100))
    c0 = rng.standard_normal((10, 100))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4)).cache_on_device()
    for agg in (False, True):
        c, _ = kmeans.kmeans(df, c0, num_iters=6, tf_aggregate=agg)
        assert np.isfinite(c).all()

    g, iname, oname = cnn.inception_v3(image_size=107, width=0.5)
    x = np.random.default_rng(1).random((24, 107, 107, 3), dtype=np.float32)
    idf = tfs.from_columns({iname: x}, num_partitions=2)
    probs = tfs.map_blocks(g.get_tensor_by_name(oname + ":0"), idf, trim=True).to_numpy(oname)
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-4)

    s1 = _C.device_pool_stats()
    assert s1["allocs"] > s0["allocs"]  # the workloads did allocate through the pool
    assert s1["fallbacks"] == s0["fallbacks"], (s0, s1)

"""Whole-model numerics on the GPU: the frozen CNN graphs (implicit-GEMM conv,
pooling, concat, softmax, top-k) and K-Means executed by the HIP kernels,
compared with the same graphs run by the host (ATen) executor."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd.models import cnn, kmeans  # noqa: E402


def _run(g, fetches, iname, x, dev):
    prog = engine.program(g.serialize(), fetches, [iname])
    return [o.cpu() for o in engine.run_program(prog, [torch.from_numpy(x)], dev)]


@pytest.mark.parametrize("builder,size,width", [(cnn.inception_v3, 75, 0.25), (cnn.inception_v3, 107, 0.5),
                                                (cnn.vgg16, 32, 0.25)])
def test_cnn_gpu_matches_host(builder, size, width):
    kw = dict(image_size=size, width=width)
    if builder is cnn.vgg16:
        kw["fc_width"] = 64
    g, iname, oname = builder(**kw)
    vals, idx = cnn.top_k_classes(g, oname, k=5)
    x = np.random.default_rng(0).random((3, size, size, 3), dtype=np.float32)
    fetches = [oname, vals.op.name, idx.op.name]
    gpu = _run(g, fetches, iname, x, torch.device("cuda", 0))
    cpu = _run(g, fetches, iname, x, torch.device("cpu"))
    torch.testing.assert_close(gpu[0], cpu[0], rtol=2e-3, atol=2e-5)
    assert torch.allclose(gpu[0].sum(1), torch.ones(3), atol=1e-4)


def test_inception_map_blocks_device_frame():
    g, iname, oname = cnn.inception_v3(image_size=75, width=0.25)
    x = np.random.default_rng(1).random((10, 75, 75, 3), dtype=np.float32)
    df = tfs.from_columns({iname: x}, num_partitions=3).cache_on_device()
    out = tfs.map_blocks(g.get_tensor_by_name(oname + ":0"), df, trim=True)
    assert out.count() == 10
    probs = out.to_numpy(oname)
    assert probs.shape == (10, 1000)
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-4)


def test_kmeans_gpu_matches_numpy():
    rng = np.random.default_rng(5)
    pts = rng.uniform(0, 1, (20000, 100))
    c0 = rng.standard_normal((10, 100))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4))
    c1, d1 = kmeans.run_one_step(df, c0)
    c2, d2 = kmeans.run_one_step2(df, c0)
    want_c, want_d = kmeans.numpy_step(pts, c0)
    np.testing.assert_allclose(c1, want_c, rtol=1e-9, atol=1e-9)
    assert abs(d1 - want_d) < 1e-6 * want_d and abs(d2 - want_d) < 1e-6 * want_d

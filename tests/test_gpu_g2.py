"""The g2 f32 MFMA core (csrc/kernels/gemm_g2_core.h: one wave per SIMD,
LDS-DMA staging) against an fp64 host reference, every g2 tile forced in turn:
plain GEMMs with B [K][N] and B^T [N][K] (transpose_b), M / N / K tails that
fall inside a tile, bias + ReLU in the vector epilogue and a transcendental
activation (heavy epilogue), split-K (small grids), batched GEMMs, and the
implicit-GEMM conv (SAME / VALID padding, strides, 1x7 / 7x1 taps, channel
counts that leave N tails). The error is measured relative to sum|a*b| per
output. Bit-identity with the round-4 core's tiles is
tests/test_gpu_precision.py::test_every_f32_tile_gives_bitwise_identical_results.
Reference workloads: BASELINE config 3 (MatMul+Relu) and config 5
(Inception-v3 convs, reference src/main/python/tensorframes_snippets/read_image.py:62-118)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

DEV = torch.device("cuda", 0)
FIRST_G2 = 22
G2_TILES = list(range(FIRST_G2, _C.gemm_tile_count()))


def run(g, fetches, feeds):
    names = list(feeds)
    prog = engine.program(g.serialize(), fetches, names)
    ins = [torch.as_tensor(np.asarray(feeds[n])) for n in names]
    return [o.cpu().numpy() for o in engine.run_program(prog, ins, DEV)]


@pytest.fixture
def forced():
    def force(cfg):
        _C.set_gemm_tile(cfg)
    yield force
    _C.set_gemm_tile(-1)


def test_g2_tiles_exist():
    assert len(G2_TILES) == 11
    assert tuple(_C.gemm_tile_dims(G2_TILES[-1])[:2]) == (128, 224)


@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(1000, 192, 720), (4099, 260, 300), (600, 64, 2048), (70000, 100, 64)])
def test_g2_gemm_matches_fp64(forced, tb, shape):
    m, n, k = shape
    rng = np.random.default_rng(m + n + k)
    x = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    w = rng.uniform(-1, 1, (n, k) if tb else (k, n)).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, k], name="x")
        mm = tf.matmul(xi, tf.constant(w), transpose_b=tb)
        tf.nn.relu(tf.nn.bias_add(mm, tf.constant(b)), name="y")
        tf.tanh(mm, name="t")  # heavy epilogue (transcendental activation)
    wt = w.T if tb else w
    ref = x.astype(np.float64) @ wt.astype(np.float64)
    scale = np.abs(x).astype(np.float64) @ np.abs(wt).astype(np.float64)
    for cfg in G2_TILES:
        forced(cfg)
        y, t = run(g, ["y", "t"], {"x": x})
        err = np.max(np.abs(y - np.maximum(ref + b, 0)) / (scale + 1.0))
        assert err < 2e-6, f"tile {cfg}: {err}"
        assert np.max(np.abs(t - np.tanh(ref)) / (scale + 1.0)) < 4e-6, f"tile {cfg}"


def test_g2_batched_matmul(forced):
    rng = np.random.default_rng(3)
    a = rng.uniform(-1, 1, (3, 300, 96)).astype(np.float32)
    b = rng.uniform(-1, 1, (3, 96, 128)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        ai = tf.placeholder(tf.float32, [3, 300, 96], name="a")
        tf.matmul(ai, tf.constant(b), name="y")
    want = np.einsum("bmk,bkn->bmn", a.astype(np.float64), b.astype(np.float64))
    for cfg in (FIRST_G2, FIRST_G2 + 4):
        forced(cfg)
        (y,) = run(g, ["y"], {"a": a})
        assert np.max(np.abs(y - want)) < 1e-4, cfg


CONVS = [  # N, H, W, C, KH, KW, OC, stride, padding
    (8, 25, 25, 48, 5, 5, 64, 1, "SAME"),
    (4, 52, 52, 80, 3, 3, 192, 1, "VALID"),
    (8, 25, 25, 288, 3, 3, 384, 2, "VALID"),
    (16, 12, 12, 128, 1, 7, 192, 1, "SAME"),
    (16, 12, 12, 160, 7, 1, 160, 1, "SAME"),
    (32, 5, 5, 448, 3, 3, 384, 1, "SAME"),
    (4, 13, 11, 36, 3, 3, 52, 2, "SAME"),
]


@pytest.mark.parametrize("geom", CONVS)
def test_g2_conv_matches_fp64(forced, geom):
    nb, h, w, c, kh, kw, oc, s, pad = geom
    rng = np.random.default_rng(h * w + c)
    x = rng.uniform(-1, 1, (nb, h, w, c)).astype(np.float32)
    f = rng.uniform(-1, 1, (kh, kw, c, oc)).astype(np.float32)
    bias = rng.uniform(-1, 1, oc).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, h, w, c], name="x")
        cv = tf.nn.conv2d(xi, tf.constant(f), [1, s, s, 1], pad)
        tf.nn.relu(tf.nn.bias_add(cv, tf.constant(bias)), name="y")
    xt = torch.from_numpy(x).double().permute(0, 3, 1, 2)
    ft = torch.from_numpy(f).double().permute(3, 2, 0, 1)
    if pad == "SAME":
        oh, ow = -(-h // s), -(-w // s)
        ph, pw = max((oh - 1) * s + kh - h, 0), max((ow - 1) * s + kw - w, 0)
        xt = torch.nn.functional.pad(xt, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    ref = torch.nn.functional.conv2d(xt, ft, stride=s).permute(0, 2, 3, 1).numpy()
    scale = torch.nn.functional.conv2d(xt.abs(), ft.abs(), stride=s).permute(0, 2, 3, 1).numpy()
    want = np.maximum(ref + bias, 0)
    for cfg in G2_TILES:
        forced(cfg)
        (y,) = run(g, ["y"], {"x": x})
        assert y.shape == want.shape
        err = np.max(np.abs(y - want) / (scale + 1.0))
        assert err < 2e-6, f"tile {cfg}: {err}"

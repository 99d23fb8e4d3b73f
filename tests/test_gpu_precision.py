"""Reduced-precision compute modes of float32 MatMul / Conv2D (Config.precision,
kernels/gemm_bf16.hip) against an fp64 host reference. The error is measured
relative to sum|a*b| per output (the scale of the rounding of each product):
bf16x3 keeps ~16 operand bits, bf16 8 bits. Also checks the default mode is
still the exact-f32 MFMA core and that switching modes takes effect."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

DEV = torch.device("cuda", 0)
TOL = {"f32": 2e-6, "bf16x3": 1e-4, "bf16": 2e-2}


@pytest.fixture(autouse=True)
def restore_precision():
    yield
    tfs.set_config(precision="f32")


def run(g, fetches, feeds):
    names = list(feeds)
    prog = engine.program(g.serialize(), fetches, names)
    ins = [torch.as_tensor(np.asarray(feeds[n])) for n in names]
    return [o.cpu().numpy() for o in engine.run_program(prog, ins, DEV)]


def rel_err(got, want, scale):
    return float(np.max(np.abs(got - want) / (scale + 1e-30)))


@pytest.mark.parametrize("mode", ["f32", "bf16x3", "bf16"])
@pytest.mark.parametrize("shape", [(1000, 96, 128), (4099, 130, 300), (64, 8, 1024)])
def test_matmul_bias_relu_modes(mode, shape):
    m, n, k = shape
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    w = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    tfs.set_config(precision=mode)
    assert _C.f32_precision() == {"f32": 0, "bf16": 1, "bf16x3": 2}[mode]
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, k], name="x")
        tf.nn.bias_add(tf.matmul(xi, tf.constant(w)), tf.constant(b), name="lin")
    (got,) = run(g, ["lin"], {"x": x})
    want = x.astype(np.float64) @ w.astype(np.float64) + b
    scale = np.abs(x.astype(np.float64)) @ np.abs(w.astype(np.float64)) + np.abs(b)
    assert rel_err(got, want, scale) < TOL[mode]


@pytest.mark.parametrize("mode", ["bf16x3", "bf16"])
@pytest.mark.parametrize("geom", [(2, 17, 19, 8, 3, 3, 24, 1, "SAME"), (3, 15, 15, 12, 5, 5, 40, 2, "VALID"),
                                  (2, 9, 9, 64, 1, 1, 72, 1, "SAME"), (2, 12, 12, 16, 1, 7, 20, 1, "SAME")])
def test_conv2d_modes(mode, geom):
    n, h, w_, c, kh, kw, oc, s, pad = geom
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, (n, h, w_, c)).astype(np.float32)
    f = rng.uniform(-1, 1, (kh, kw, c, oc)).astype(np.float32)
    tfs.set_config(precision=mode)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, h, w_, c], name="x")
        tf.nn.relu(tf.nn.conv2d(xi, tf.constant(f), [1, s, s, 1], pad), name="y")
    (got,) = run(g, ["y"], {"x": x})
    xt = torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2)
    ft = torch.as_tensor(f, dtype=torch.float64).permute(3, 2, 0, 1)
    if pad == "SAME":
        oh, ow = -(-h // s), -(-w_ // s)
        ph, pw = max(0, (oh - 1) * s + kh - h), max(0, (ow - 1) * s + kw - w_)
        xt = torch.nn.functional.pad(xt, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    want = torch.relu(torch.nn.functional.conv2d(xt, ft, stride=s)).permute(0, 2, 3, 1).numpy()
    scale = torch.nn.functional.conv2d(xt.abs(), ft.abs(), stride=s).permute(0, 2, 3, 1).numpy()
    assert got.shape == want.shape
    assert rel_err(got, want, scale) < TOL[mode]


def test_bf16_is_faster_than_f32_on_a_big_gemm():
    """The bf16x3 path really ran: same GEMM, measurably different time and a
    non-zero (but tiny) deviation from the exact-f32 result."""
    rng = np.random.default_rng(3)
    x = torch.as_tensor(rng.uniform(-1, 1, (262144, 512)).astype(np.float32), device=DEV)
    w = rng.uniform(-1, 1, (512, 512)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, 512], name="x")
        tf.matmul(xi, tf.constant(w), name="y")
    res = {}
    for mode in ("f32", "bf16x3"):
        tfs.set_config(precision=mode)
        prog = engine.program(g.serialize(), ["y"], ["x"])
        engine.run_program(prog, [x], DEV)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            (y,) = engine.run_program(prog, [x], DEV)
        e.record()
        torch.cuda.synchronize()
        res[mode] = (s.elapsed_time(e) / 5, y)
    diff = (res["f32"][1] - res["bf16x3"][1]).abs().max().item()
    assert 0 < diff < 1e-2
    assert res["bf16x3"][0] < res["f32"][0]


def test_every_f32_tile_gives_bitwise_identical_results():
    """The tile autotuner may pick any single-pass tile of the f32 core: every
    tile sums each output's K products in the same order (BK=16 LDS steps of
    32x32x2 MFMAs), so the results are bit-identical whichever tile wins.
    (Shapes sized so every forced tile stays single-pass: a split-K plan sums in
    another order, and the tuner never picks one.)"""
    rng = np.random.default_rng(9)
    # >= 256 row tiles of the tallest (256-row) tiles: no forced tile goes split-K
    x = rng.uniform(-1, 1, (70000, 300)).astype(np.float32)
    w = rng.uniform(-1, 1, (300, 256)).astype(np.float32)
    img = rng.uniform(-1, 1, (176, 20, 20, 32)).astype(np.float32)
    f = rng.uniform(-1, 1, (3, 3, 32, 192)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, 300], name="x")
        tf.matmul(xi, tf.constant(w), name="y")
        ii = tf.placeholder(tf.float32, [None, 20, 20, 32], name="img")
        tf.nn.conv2d(ii, tf.constant(f), [1, 1, 1, 1], "SAME", name="c")
    outs = {}
    try:
        for cfg in range(_C.gemm_tile_count()):
            _C.set_gemm_tile(cfg)
            outs[cfg] = run(g, ["y", "c"], {"x": x, "img": img})
    finally:
        _C.set_gemm_tile(-1)
    auto = run(g, ["y", "c"], {"x": x, "img": img})
    for cfg, (y, c) in outs.items():
        assert np.array_equal(y, outs[0][0]), f"tile {cfg}: GEMM differs"
        assert np.array_equal(c, outs[0][1]), f"tile {cfg}: conv differs"
    assert np.array_equal(auto[0], outs[0][0]) and np.array_equal(auto[1], outs[0][1])

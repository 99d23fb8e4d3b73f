"""3x3 VALID MaxPool -> 1x1 conv (+ bias + ReLU) fused into one kernel
(csrc/kernels/conv_smallc.hip pool_conv1x1, planner pass "pool_conv" in
csrc/runtime/executor.cpp): Inception-v3 MaxPool_3a -> Conv2d_3b. The fused
step must give the unfused plan's bits (same k order as the GEMM cores) and
match a float64 host reference of the same ops."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

DEV = torch.device("cuda", 0)

CASES = [  # n, h, w, c, oc, stride, relu
    (4, 27, 27, 64, 80, 2, True),   # Inception MaxPool_3a -> Conv2d_3b (109 -> 54 at 224)
    (3, 20, 17, 32, 40, 2, False),  # OC tail, odd sizes
    (2, 9, 11, 16, 96, 1, True),    # stride-1 pool, three 32-oc tiles
    (1, 7, 7, 64, 7, 3, True),      # tiny OC, one partial pixel group
]


def _graph(h, w, c, f, b, stride, relu):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, h, w, c], name="x")
        p = tf.nn.max_pool(x, [1, 3, 3, 1], [1, stride, stride, 1], "VALID")
        y = tf.nn.bias_add(tf.nn.conv2d(p, tf.constant(f), [1, 1, 1, 1], "VALID"), tf.constant(b))
        tf.identity(tf.nn.relu(y) if relu else y, name="y")
    return g


def _run(g, x, fused):
    engine.clear_program_cache()
    _C.set_pool_conv_fusion(fused)
    try:
        prog = engine.program(g.serialize(), ["y"], ["x"])
        desc = prog.describe([torch.from_numpy(x[:1])], True)
        y = engine.run_program(prog, [torch.from_numpy(x)], DEV)[0].cpu().numpy()
    finally:
        _C.set_pool_conv_fusion(True)
        engine.clear_program_cache()
    return desc, y


@pytest.mark.parametrize("case", CASES)
def test_pool_conv_fused_bitwise_and_fp64(case):
    n, h, w, c, oc, s, relu = case
    rng = np.random.default_rng(n * h + c + oc)
    x = rng.uniform(-1, 1, (n, h, w, c)).astype(np.float32)
    f = rng.uniform(-1, 1, (1, 1, c, oc)).astype(np.float32)
    b = rng.uniform(-1, 1, oc).astype(np.float32)
    g = _graph(h, w, c, f, b, s, relu)
    d_on, y_on = _run(g, x, True)
    d_off, y_off = _run(g, x, False)
    assert "+maxpool3x3/" in d_on and "+maxpool3x3/" not in d_off
    assert np.array_equal(y_on, y_off), "fused pool -> 1x1 conv differs from the unfused plan"
    ph, pw = (h - 3) // s + 1, (w - 3) // s + 1
    xp = np.stack([x[:, dy:dy + s * (ph - 1) + 1:s, dx:dx + s * (pw - 1) + 1:s] for dy in range(3) for dx in range(3)])
    pooled = xp.max(0).astype(np.float64)
    want = pooled @ f[0, 0].astype(np.float64) + b
    if relu:
        want = np.maximum(want, 0)
    scale = np.abs(pooled) @ np.abs(f[0, 0].astype(np.float64)) + np.abs(b)
    assert y_on.shape == want.shape
    assert np.max(np.abs(y_on - want) / scale) < 1e-6


def test_fused_kernel_runs(tmp_path):
    """The step runs the fused kernel (its label), not the pool-into-a-temporary fallback."""
    from tensorframes_amd.utils.profiling import step_profile
    rng = np.random.default_rng(5)
    f = rng.uniform(-1, 1, (1, 1, 64, 80)).astype(np.float32)
    g = _graph(27, 27, 64, f, np.zeros(80, np.float32), 2, True)
    engine.clear_program_cache()
    _C.set_pool_conv_fusion(True)
    try:
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn(4, 27, 27, 64, device=DEV)
        engine.run_program(prog, [xin], DEV)
        torch.cuda.synchronize()
        rows = step_profile(lambda: engine.run_program(prog, [xin], DEV), str(tmp_path / "p.json"), "t")
    finally:
        _C.set_pool_conv_fusion(True)
        engine.clear_program_cache()
    conv = [r for r in rows if r["op"] == "Conv2D"]
    assert len(conv) == 1 and conv[0]["algo"] == "maxpool3x3+conv1x1", rows
    assert not any(r["op"] == "MaxPool" for r in rows)


def test_inception_plan_fuses_maxpool_3a():
    """The full Inception-v3 plan runs MaxPool_3a inside Conv2d_3b's step."""
    from tensorframes_amd.models import cnn
    g, iname, oname = cnn.inception_v3(image_size=224)
    _C.set_pool_conv_fusion(True)
    try:
        engine.clear_program_cache()
        prog = engine.program(g.serialize(), [oname], [iname])
        desc = prog.describe([torch.zeros((1, 224, 224, 3))], True)
    finally:
        _C.set_pool_conv_fusion(True)
        engine.clear_program_cache()
    assert "+maxpool3x3/2-in" in desc

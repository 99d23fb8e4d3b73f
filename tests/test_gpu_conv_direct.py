"""Direct narrow conv (csrc/kernels/conv_direct.hip: C in {32, 64}, OC <= 64,
wide images; filter in LDS, A straight to registers) against an fp64 host
reference of the same op, against the implicit-GEMM core (same values to f32
rounding; the kernel sums k in a different fixed order), and run-to-run
bitwise stable."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

from test_gpu_conv_smallc import conv_ref  # noqa: E402

DEV = torch.device("cuda", 0)

CASES = [  # n, h, w, c, kh, kw, oc, stride, pad, dil, relu
    (2, 70, 70, 32, 3, 3, 32, 1, "VALID", 1, True),   # Inception Conv2d_2a shape class
    (2, 67, 67, 32, 3, 3, 64, 1, "SAME", 1, True),    # Conv2d_2b
    (1, 66, 70, 64, 3, 3, 64, 1, "SAME", 1, False),   # VGG conv1_2 class, C = 64
    (1, 130, 130, 32, 3, 3, 48, 2, "SAME", 1, True),  # stride 2, OC not a multiple of 32
    (1, 72, 72, 32, 2, 3, 20, 1, "SAME", 2, True),    # dilation, odd filter
]


@pytest.mark.parametrize("case", CASES)
def test_direct_conv_matches_fp64_and_gemm_core(case):
    n, h, w, c, kh, kw, oc, s, pad, dil, relu = case
    rng = np.random.default_rng(sum(case[:7]))
    x = rng.uniform(-1, 1, (n, h, w, c)).astype(np.float32)
    f = (rng.uniform(-1, 1, (kh, kw, c, oc)) / np.sqrt(kh * kw * c)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, oc).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, h, w, c], name="x")
        y = tf.nn.conv2d(xi, tf.constant(f), [1, s, s, 1], pad, dilations=[1, dil, dil, 1])
        y = tf.nn.bias_add(y, tf.constant(b))
        tf.identity(tf.nn.relu(y) if relu else y, name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    xt = torch.from_numpy(x)
    try:
        _C.set_conv_direct(True)
        d1 = engine.run_program(prog, [xt], DEV)[0].cpu().numpy()
        d2 = engine.run_program(prog, [xt], DEV)[0].cpu().numpy()
        _C.set_conv_direct(False)
        core = engine.run_program(prog, [xt], DEV)[0].cpu().numpy()
    finally:
        _C.set_conv_direct(True)
    assert np.array_equal(d1, d2), "direct conv is not run-to-run stable"
    want = conv_ref(x.astype(np.float64), f.astype(np.float64), b, s, pad, dil, relu)
    np.testing.assert_allclose(d1, want, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(d1, core, rtol=1e-5, atol=2e-5)


def test_direct_three_column_tiles():
    """OC = 80: three 32-column tiles, the last one partial (1x2 filter, C = 64)."""
    rng = np.random.default_rng(11)
    n, h, w, c, oc = 8, 70, 70, 64, 80
    x = rng.uniform(-1, 1, (n, h, w, c)).astype(np.float32)
    f = (rng.uniform(-1, 1, (1, 2, c, oc)) / 11).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, oc).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, h, w, c], name="x")
        tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(xi, tf.constant(f), [1, 1, 1, 1], "VALID"), tf.constant(b)), name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    xt = torch.from_numpy(x)
    try:
        _C.set_conv_direct(True)
        d = engine.run_program(prog, [xt], DEV)[0].cpu().numpy()
        _C.set_conv_direct(False)
        core = engine.run_program(prog, [xt], DEV)[0].cpu().numpy()
    finally:
        _C.set_conv_direct(True)
    want = conv_ref(x.astype(np.float64), f.astype(np.float64), b, 1, "VALID", 1, True)
    np.testing.assert_allclose(d, want, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(d, core, rtol=1e-5, atol=2e-5)

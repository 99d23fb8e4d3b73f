"""Direct small-reduction conv (csrc/kernels/conv_smallc.hip, KH*KW*C <= 32:
RGB stems) against the implicit-GEMM core (bitwise: same k order) and an fp64
host reference of the same op. The SAME cases run the padded fast path (32-bit
offsets, per-tap bounds test), the in-bounds VALID ones the unpadded one."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

DEV = torch.device("cuda", 0)


def conv_ref(x, w, b, stride, pad, dil, relu):
    """fp64 NHWC conv with TF SAME/VALID padding."""
    n, h, wd, c = x.shape
    kh, kw, _, oc = w.shape
    ekh, ekw = (kh - 1) * dil + 1, (kw - 1) * dil + 1
    if pad == "SAME":
        oh, ow = -(-h // stride), -(-wd // stride)
        ph = max((oh - 1) * stride + ekh - h, 0)
        pw = max((ow - 1) * stride + ekw - wd, 0)
        pt, pl = ph // 2, pw // 2
    else:
        oh, ow = (h - ekh) // stride + 1, (wd - ekw) // stride + 1
        pt = pl = ph = pw = 0
    xp = np.zeros((n, h + ph, wd + pw, c))
    xp[:, pt:pt + h, pl:pl + wd] = x
    y = np.zeros((n, oh, ow, oc))
    for i in range(kh):
        for j in range(kw):
            patch = xp[:, i * dil:i * dil + stride * (oh - 1) + 1:stride, j * dil:j * dil + stride * (ow - 1) + 1:stride]
            y += patch @ w[i, j].astype(np.float64)
    y += b
    return np.maximum(y, 0) if relu else y


CASES = [  # n, h, w, c, kh, kw, oc, stride, pad, dil, relu
    (8, 37, 41, 3, 3, 3, 32, 2, "VALID", 1, True),    # Inception Conv2d_1a
    (4, 30, 30, 3, 3, 3, 64, 1, "SAME", 1, True),     # VGG conv1_1 (padded fast path)
    (3, 17, 19, 1, 5, 5, 20, 1, "SAME", 1, False),    # odd OC, one channel
    (2, 23, 23, 2, 3, 3, 48, 1, "SAME", 2, True),     # dilation
    (5, 9, 9, 4, 2, 2, 7, 3, "SAME", 1, False),       # stride 3, tiny OC
    (1, 7, 5, 3, 1, 3, 33, 1, "VALID", 1, True),      # M not a multiple of 32
    (3, 19, 21, 3, 3, 3, 40, 2, "VALID", 1, False),   # in-bounds fast path, no activation
    (2, 16, 16, 2, 2, 2, 32, 2, "VALID", 2, True),    # fast path with dilation
]


def _run(case):
    n, h, w, c, kh, kw, oc, s, pad, dil, relu = case
    rng = np.random.default_rng(sum(case[:7]))
    x = rng.uniform(-1, 1, (n, h, w, c)).astype(np.float32)
    f = rng.uniform(-1, 1, (kh, kw, c, oc)).astype(np.float32)
    b = rng.uniform(-1, 1, oc).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, h, w, c], name="x")
        y = tf.nn.conv2d(xi, tf.constant(f), [1, s, s, 1], pad, dilations=[1, dil, dil, 1])
        y = tf.nn.bias_add(y, tf.constant(b))
        tf.identity(tf.nn.relu(y) if relu else y, name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    outs = {}
    try:
        for on in (True, False):
            _C.set_conv_smallc(on)
            outs[on] = engine.run_program(prog, [torch.from_numpy(x)], DEV)[0].cpu().numpy()
    finally:
        _C.set_conv_smallc(True)
    return x, f, b, outs


@pytest.mark.parametrize("case", CASES)
def test_smallc_matches_gemm_core_bitwise_and_fp64(case):
    n, h, w, c, kh, kw, oc, s, pad, dil, relu = case
    x, f, b, outs = _run(case)
    assert np.array_equal(outs[True], outs[False]), "direct small-C conv differs from the implicit-GEMM core"
    want = conv_ref(x.astype(np.float64), f.astype(np.float64), b, s, pad, dil, relu)
    np.testing.assert_allclose(outs[True], want, rtol=1e-5, atol=1e-5)

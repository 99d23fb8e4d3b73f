"""Winograd F(2x2,3x3) conv path, host side (no GPU): the planner's filter
transform (conv_wino_filter, fp64 -> f32, layout [C/8][16][2][OCP][4]) driven
through a numpy emulation of exactly the kernel's algorithm (B^T d B per wave
row, M = sum_c V U, A^T M A) must reproduce a float64 direct convolution, and
a GPU plan must carry one Winograd filter per distinct 3x3 stride-1 filter.
The kernel itself: tests/test_gpu_wino.py. Reference workload: BASELINE
config 5, src/main/python/tensorframes_snippets/read_image.py:62-71."""
import numpy as np
import pytest

from tensorframes_amd import engine, tf
from tensorframes_amd._native import _C

BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)


def direct(x, f, pad):
    n, h, w, c = x.shape
    oc = f.shape[3]
    p = 1 if pad == "SAME" else 0
    xp = np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))
    oh, ow = h + 2 * p - 2, w + 2 * p - 2
    y = np.zeros((n, oh, ow, oc))
    for a in range(3):
        for b in range(3):
            y += np.einsum("nhwc,co->nhwo", xp[:, a:a + oh, b:b + ow, :], f[a, b])
    return y


def emulate(x, u_flat, oc, pad):
    n, h, w, c = x.shape
    ocp = -(-oc // 64) * 64
    u = u_flat.astype(np.float64).reshape(c // 8, 16, 2, ocp, 4).transpose(1, 0, 2, 4, 3).reshape(16, c, ocp)
    p = 1 if pad == "SAME" else 0
    oh, ow = h + 2 * p - 2, w + 2 * p - 2
    th, tw = -(-oh // 2), -(-ow // 2)
    # zero padding that covers the patch of every (partial) edge tile
    xp = np.zeros((n, 2 * th + 2, 2 * tw + 2, c))
    xp[:, p:p + h, p:p + w, :] = x
    y = np.zeros((n, 2 * th, 2 * tw, oc))
    for ty in range(th):
        for tx in range(tw):
            d = xp[:, 2 * ty:2 * ty + 4, 2 * tx:2 * tx + 4, :]            # n, 4, 4, c
            v = np.einsum("ia,nabc,jb->nijc", BT, d, BT).reshape(n, 16, c)
            m = np.einsum("nxc,xco->nxo", v, u)[:, :, :oc].reshape(n, 4, 4, oc)
            y[:, 2 * ty:2 * ty + 2, 2 * tx:2 * tx + 2, :] = np.einsum("pi,nijo,qj->npqo", AT, m, AT)
    return y[:, :oh, :ow, :]


@pytest.mark.parametrize("geom", [(2, 6, 6, 8, 8, "SAME"), (1, 7, 9, 8, 12, "VALID"), (2, 5, 5, 24, 68, "SAME")])
def test_filter_transform_and_algorithm_match_direct(geom):
    n, h, w, c, oc, pad = geom
    rng = np.random.default_rng(h * w + c)
    x = rng.uniform(-1, 1, (n, h, w, c))
    f = rng.uniform(-1, 1, (3, 3, c, oc)).astype(np.float32)
    import torch
    u = _C.conv_wino_filter(torch.from_numpy(f)).numpy()
    assert u.shape == (16 * c * (-(-oc // 64) * 64),)
    want = direct(x, f.astype(np.float64), pad)
    got = emulate(x, u, oc, pad)
    scale = direct(np.abs(x), np.abs(f.astype(np.float64)), pad)
    assert np.max(np.abs(got - want) / (scale + 1)) < 1e-6


def test_filter_padding_is_zero():
    import torch
    f = np.ones((3, 3, 8, 10), np.float32)
    u = _C.conv_wino_filter(torch.from_numpy(f)).numpy().reshape(1, 16, 2, 64, 4)
    assert np.all(u[:, :, :, 10:, :] == 0)
    # xi (0,0) is g[0][0]; xi (1,1) is (sum over the 3x3) / 4
    assert np.allclose(u[0, 0, :, :10], 1.0)
    assert np.allclose(u[0, 5, :, :10], 9 / 4)


def _inception_like_graph():
    rng = np.random.default_rng(0)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 9, 9, 8], name="x")
        a = tf.nn.relu(tf.nn.conv2d(x, tf.constant(rng.uniform(-1, 1, (3, 3, 8, 16)).astype(np.float32)),
                                    [1, 1, 1, 1], "SAME"))
        b = tf.nn.conv2d(a, tf.constant(rng.uniform(-1, 1, (3, 3, 16, 12)).astype(np.float32)), [1, 2, 2, 1], "VALID")
        c = tf.nn.conv2d(a, tf.constant(rng.uniform(-1, 1, (1, 1, 16, 4)).astype(np.float32)), [1, 1, 1, 1], "SAME")
        tf.identity(b, name="b")
        tf.identity(c, name="c")
    return g


def test_gpu_plan_carries_winograd_filters_only_for_3x3_stride1():
    import torch
    g = _inception_like_graph()
    prog = engine.program(g.serialize(), ["b", "c"], ["x"])
    desc = prog.describe([torch.zeros(2, 9, 9, 8)], True)
    assert "1 Winograd filters" in desc, desc
    assert desc.count("+winograd") == 1, desc
    # host plans never carry one; with the switch off GPU plans do not either
    assert "+winograd" not in prog.describe([torch.zeros(2, 9, 9, 8)], False)
    _C.set_conv_wino(False)
    try:
        assert "+winograd" not in prog.describe([torch.zeros(2, 9, 9, 8)], True)
    finally:
        _C.set_conv_wino(True)

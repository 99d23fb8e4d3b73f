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
    f = np.ones((3, 3, 8, 12), np.float32)
    u = _C.conv_wino_filter(torch.from_numpy(f)).numpy().reshape(1, 16, 2, 64, 4)
    assert np.all(u[:, :, :, 12:, :] == 0)
    # xi (0,0) is g[0][0]; xi (1,1) is (sum over the 3x3) / 4
    assert np.allclose(u[0, 0, :, :12], 1.0)
    assert np.allclose(u[0, 5, :, :12], 9 / 4)


def emulate27(x, u_flat, oc, axis):
    """The F(2,7) kernel's algorithm (its exact input-transform formulas) on a
    1x7 (axis 0, along W) or 7x1 (axis 1, along H) SAME conv."""
    n, h, w, c = x.shape
    ocp = -(-oc // 64) * 64
    u = u_flat.astype(np.float64).reshape(c // 8, 8, 2, ocp, 4).transpose(1, 0, 2, 4, 3).reshape(8, c, ocp)[:, :, :oc]
    xs = x if axis == 0 else x.transpose(0, 2, 1, 3)      # conv along the W axis of xs
    L = xs.shape[2]
    nt = -(-L // 2)
    xp = np.zeros((n, xs.shape[1], 2 * nt + 6, c))
    xp[:, :, 3:3 + L, :] = xs
    y = np.zeros((n, xs.shape[1], 2 * nt, oc))
    for t in range(nt):
        d = [xp[:, :, 2 * t + p, :] for p in range(8)]
        v = [None] * 8
        v[0] = (d[6] - d[0]) + 5.25 * (d[2] - d[4])
        v[7] = (d[7] - d[1]) + 5.25 * (d[3] - d[5])
        e1, o1 = (d[2] + d[6]) - 4.25 * d[4], (d[1] + d[5]) - 4.25 * d[3]
        v[1], v[2] = e1 + o1, e1 - o1
        e3, o3 = (0.25 * d[2] + d[6]) - 1.25 * d[4], (0.5 * d[1] + 2 * d[5]) - 2.5 * d[3]
        v[3], v[4] = e3 + o3, e3 - o3
        e5, o5 = (4 * d[2] + d[6]) - 5 * d[4], (2 * d[1] + 0.5 * d[5]) - 2.5 * d[3]
        v[5], v[6] = e5 + o5, e5 - o5
        m = [np.einsum("nhc,co->nho", v[i], u[i]) for i in range(8)]
        y[:, :, 2 * t] = m[0] + m[1] + m[2] + m[3] + m[4] + m[5] + m[6]
        y[:, :, 2 * t + 1] = (m[1] - m[2]) + 2 * (m[3] - m[4]) + 0.5 * (m[5] - m[6]) + m[7]
    y = y[:, :, :L]
    return y if axis == 0 else y.transpose(0, 2, 1, 3)


@pytest.mark.parametrize("axis", [0, 1])
def test_f27_transform_and_algorithm_match_direct(axis):
    import torch
    rng = np.random.default_rng(7 + axis)
    x = rng.uniform(-1, 1, (2, 6, 9, 16))
    kshape = (1, 7, 16, 12) if axis == 0 else (7, 1, 16, 12)
    f = rng.uniform(-1, 1, kshape).astype(np.float32)
    u = _C.conv_wino_filter(torch.from_numpy(f)).numpy()
    assert u.shape == (8 * 16 * 64,)
    xt = torch.from_numpy(x).permute(0, 3, 1, 2)
    ft = torch.from_numpy(f.astype(np.float64)).permute(3, 2, 0, 1)
    pad = (0, 3) if axis == 0 else (3, 0)
    want = torch.nn.functional.conv2d(xt, ft, padding=pad).permute(0, 2, 3, 1).numpy()
    got = emulate27(x, u, 12, axis)
    scale = torch.nn.functional.conv2d(xt.abs(), ft.abs(), padding=pad).permute(0, 2, 3, 1).numpy()
    assert np.max(np.abs(got - want) / (scale + 1)) < 1e-6


def test_f27_matrices_from_toom_cook():
    """The kernel's B^T / A^T and the host's G7 reproduce 1-D correlation for
    every (d, g): sum_i A^T[j][i] G[i][k] B^T[i][l] == [l == j + k]."""
    from fractions import Fraction as F
    G7 = [[-1, 0, 0, 0, 0, 0, 0], [F(-2, 9)] * 7, [F(-2, 9) * (-1) ** k for k in range(7)],
          [F(1, 90) * 2 ** k for k in range(7)], [F(1, 90) * (-2) ** k for k in range(7)],
          [F(32, 45) / 2 ** k for k in range(7)], [F(32, 45) * F(-1, 2) ** k for k in range(7)],
          [0, 0, 0, 0, 0, 0, 1]]
    BT = [[-1, 0, F(21, 4), 0, F(-21, 4), 0, 1, 0], [0, 1, 1, F(-17, 4), F(-17, 4), 1, 1, 0],
          [0, -1, 1, F(17, 4), F(-17, 4), -1, 1, 0], [0, F(1, 2), F(1, 4), F(-5, 2), F(-5, 4), 2, 1, 0],
          [0, F(-1, 2), F(1, 4), F(5, 2), F(-5, 4), -2, 1, 0], [0, 2, 4, F(-5, 2), -5, F(1, 2), 1, 0],
          [0, -2, 4, F(5, 2), -5, F(-1, 2), 1, 0], [0, -1, 0, F(21, 4), 0, F(-21, 4), 0, 1]]
    AT = [[1, 1, 1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, F(1, 2), F(-1, 2), 1]]
    for j in range(2):
        for k in range(7):
            for l in range(8):
                v = sum(F(AT[j][i]) * F(G7[i][k]) * F(BT[i][l]) for i in range(8))
                assert v == (1 if l == j + k else 0), (j, k, l, v)


def emulate45(x, u_flat, oc, pad):
    """The F(4,5) x 5-row kernel's algorithm (the F(2,7) input transform, the
    4-output A^T, rows accumulated in the transform domain) on a 5x5 conv."""
    n, h, w, c = x.shape
    ocp = -(-oc // 64) * 64
    u = (u_flat.astype(np.float64).reshape(5, c // 8, 8, 2, ocp, 4).transpose(0, 2, 1, 3, 5, 4)
         .reshape(5, 8, c, ocp)[..., :oc])
    p = 2 if pad == "SAME" else 0
    oh, ow = h + 2 * p - 4, w + 2 * p - 4
    nt = -(-ow // 4)
    xp = np.zeros((n, h + 2 * p, 4 * nt + 4, c))
    xp[:, p:p + h, p:p + w] = x
    y = np.zeros((n, oh, 4 * nt, oc))
    for t in range(nt):
        m = [0.0] * 8
        for kh in range(5):
            d = [xp[:, kh:kh + oh, 4 * t + q, :] for q in range(8)]
            v = [None] * 8
            v[0] = (d[6] - d[0]) + 5.25 * (d[2] - d[4])
            v[7] = (d[7] - d[1]) + 5.25 * (d[3] - d[5])
            e1, o1 = (d[2] + d[6]) - 4.25 * d[4], (d[1] + d[5]) - 4.25 * d[3]
            v[1], v[2] = e1 + o1, e1 - o1
            e3, o3 = (0.25 * d[2] + d[6]) - 1.25 * d[4], (0.5 * d[1] + 2 * d[5]) - 2.5 * d[3]
            v[3], v[4] = e3 + o3, e3 - o3
            e5, o5 = (4 * d[2] + d[6]) - 5 * d[4], (2 * d[1] + 0.5 * d[5]) - 2.5 * d[3]
            v[5], v[6] = e5 + o5, e5 - o5
            m = [m[i] + np.einsum("nhc,co->nho", v[i], u[kh, i]) for i in range(8)]
        s12, s34, s56 = m[1] - m[2], m[3] - m[4], m[5] - m[6]
        a12, a34, a56 = m[1] + m[2], m[3] + m[4], m[5] + m[6]
        y[:, :, 4 * t] = m[0] + a12 + a34 + a56
        y[:, :, 4 * t + 1] = s12 + 2 * s34 + 0.5 * s56
        y[:, :, 4 * t + 2] = a12 + 4 * a34 + 0.25 * a56
        y[:, :, 4 * t + 3] = s12 + 8 * s34 + 0.125 * s56 + m[7]
    return y[:, :, :ow]


@pytest.mark.parametrize("pad", ["SAME", "VALID"])
def test_f45_transform_and_algorithm_match_direct(pad):
    import torch
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, (2, 9, 11, 16))
    f = rng.uniform(-1, 1, (5, 5, 16, 12)).astype(np.float32)
    _C.set_wino_5x5(True)  # opt-in kernel (config.wino_5x5)
    try:
        u = _C.conv_wino_filter(torch.from_numpy(f)).numpy()
    finally:
        _C.set_wino_5x5(False)
    assert u.shape == (5 * 8 * 16 * 64,)
    xt = torch.from_numpy(x).permute(0, 3, 1, 2)
    ft = torch.from_numpy(f.astype(np.float64)).permute(3, 2, 0, 1)
    p = 2 if pad == "SAME" else 0
    want = torch.nn.functional.conv2d(xt, ft, padding=p).permute(0, 2, 3, 1).numpy()
    scale = torch.nn.functional.conv2d(xt.abs(), ft.abs(), padding=p).permute(0, 2, 3, 1).numpy()
    got = emulate45(x, u, 12, pad)
    assert got.shape == want.shape
    assert np.max(np.abs(got - want) / (scale + 1)) < 1e-6


def test_f45_matrices_from_toom_cook():
    """F(4,5) on the F(2,7) points: the kernel's B^T, its 4-row A^T and the
    host's G5 (G7's first 5 columns, inf row on the last tap) reproduce 1-D
    correlation exactly."""
    from fractions import Fraction as F
    pts = [0, 1, -1, 2, -2, F(1, 2), F(-1, 2)]
    scale = [-1, F(-2, 9), F(-2, 9), F(1, 90), F(1, 90), F(32, 45), F(32, 45)]
    G5 = [[scale[i] * F(pts[i]) ** k for k in range(5)] for i in range(7)] + [[0, 0, 0, 0, 1]]
    BT = [[-1, 0, F(21, 4), 0, F(-21, 4), 0, 1, 0], [0, 1, 1, F(-17, 4), F(-17, 4), 1, 1, 0],
          [0, -1, 1, F(17, 4), F(-17, 4), -1, 1, 0], [0, F(1, 2), F(1, 4), F(-5, 2), F(-5, 4), 2, 1, 0],
          [0, F(-1, 2), F(1, 4), F(5, 2), F(-5, 4), -2, 1, 0], [0, 2, 4, F(-5, 2), -5, F(1, 2), 1, 0],
          [0, -2, 4, F(5, 2), -5, F(-1, 2), 1, 0], [0, -1, 0, F(21, 4), 0, F(-21, 4), 0, 1]]
    AT = [[F(pts[i]) ** j for i in range(7)] + [1 if j == 3 else 0] for j in range(4)]
    for j in range(4):
        for k in range(5):
            for l in range(8):
                v = sum(F(AT[j][i]) * F(G5[i][k]) * F(BT[i][l]) for i in range(8))
                assert v == (1 if l == j + k else 0), (j, k, l, v)


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


def _vgg_block(pool_k=2, extra_reader=False, h=8):
    rng = np.random.default_rng(1)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, h, h, 8], name="x")
        y = tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(x, tf.constant(rng.standard_normal((3, 3, 8, 16)).astype(np.float32)),
                                                   [1, 1, 1, 1], "SAME"), tf.constant(np.ones(16, np.float32))))
        p = tf.nn.max_pool(y, [1, pool_k, pool_k, 1], [1, 2, 2, 1], "VALID")
        out = tf.reduce_sum(p, [1, 2, 3])
        if extra_reader:
            out = out + tf.reduce_sum(y, [1, 2, 3])
        tf.identity(out, name="s")
    return g


def test_plan_fuses_2x2_maxpool_into_the_winograd_conv():
    """VGG's conv -> bias -> relu -> 2x2/2 max pool becomes one step whose
    Winograd epilogue pools (the GPU plan, built from host tensors); a 3x3
    pool, a second reader of the conv output or odd output sizes keep the
    pool step."""
    import torch

    def desc(g, h=8):
        prog = engine.program(g.serialize(), ["s"], ["x"])
        return prog.describe([torch.zeros(2, h, h, 8)], True)
    d = desc(_vgg_block())
    assert "+winograd +maxpool2x2" in d and "MaxPool" not in d.split("+maxpool2x2")[1].split("\n")[0], d
    assert "+maxpool2x2" not in desc(_vgg_block(pool_k=3))
    assert "+maxpool2x2" not in desc(_vgg_block(extra_reader=True))
    assert "+maxpool2x2" not in desc(_vgg_block(h=9), h=9)


def test_config_wino_5x5_switch():
    """config.wino_5x5 (opt-in) turns the 5x5 kind on for plans made after it."""
    import torch
    import tensorframes_amd as tfs
    f = torch.zeros((5, 5, 8, 8))
    with pytest.raises(Exception):
        _C.conv_wino_filter(f)
    tfs.set_config(wino_5x5=True)
    try:
        assert _C.conv_wino_filter(f).numel() == 5 * 8 * 8 * 64
    finally:
        tfs.set_config(wino_5x5=False)
    with pytest.raises(Exception):
        _C.conv_wino_filter(f)

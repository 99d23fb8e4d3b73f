"""BroadcastTo, DepthToSpace / SpaceToDepth, SpaceToBatchND / BatchToSpaceND
(and the TF-1.x atrous_conv2d built from them), Conv2DBackpropInput
(tf.nn.conv2d_transpose), L2Loss and the two softmax
cross-entropy ops: CPU executor against numpy / torch references; the GPU
kernels against the CPU executor (gpu-marked)."""
import numpy as np
import pytest
import torch

from tensorframes_amd import engine, tf

rng = np.random.default_rng(5)


def run(g, fetches, feeds, device=torch.device("cpu")):
    names = list(feeds)
    prog = engine.program(g.serialize(), fetches, names)
    ins = [torch.as_tensor(np.asarray(feeds[n])) for n in names]
    return [o.cpu().numpy() for o in engine.run_program(prog, ins, device)]


def d2s_ref(x, b):  # TF DepthToSpace, NHWC (DCR)
    n, h, w, c = x.shape
    co = c // (b * b)
    return x.reshape(n, h, w, b, b, co).transpose(0, 1, 3, 2, 4, 5).reshape(n, h * b, w * b, co)


def s2d_ref(x, b):
    n, h, w, c = x.shape
    return x.reshape(n, h // b, b, w // b, b, c).transpose(0, 1, 3, 2, 4, 5).reshape(n, h // b, w // b, b * b * c)


def s2b_ref(x, block, pads):
    xp = np.pad(x, [[0, 0]] + [list(p) for p in pads] + [[0, 0]] * (x.ndim - 1 - len(block)))
    n = x.shape[0]
    m = len(block)
    shp = [n]
    for i, b in enumerate(block):
        shp += [xp.shape[i + 1] // b, b]
    shp += list(xp.shape[m + 1:])
    perm = [2 + 2 * i for i in range(m)] + [0] + [1 + 2 * i for i in range(m)] + list(range(2 * m + 1, len(shp)))
    y = xp.reshape(shp).transpose(perm)
    return y.reshape([n * int(np.prod(block))] + [xp.shape[i + 1] // block[i] for i in range(m)]
                     + list(xp.shape[m + 1:]))


def graph_more():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 4, 6, 8], name="x")
        v = tf.placeholder(tf.float32, [None, 3], name="v")
        lab = tf.placeholder(tf.float32, [None, 3], name="lab")
        ids = tf.placeholder(tf.int32, [None], name="ids")
        tf.broadcast_to(tf.reshape(v, [-1, 1, 3]), [5, 4, 3], name="bc")
        tf.depth_to_space(x, 2, name="d2s")
        tf.space_to_depth(x, 2, name="s2d")
        tf.space_to_batch_nd(x, [2, 3], [[1, 1], [0, 3]], name="s2b")
        tf.batch_to_space_nd(tf.space_to_batch_nd(x, [2, 2], [[0, 2], [2, 0]]), [2, 2], [[0, 2], [2, 0]], name="b2s")
        tf.nn.l2_loss(x, name="l2")
        tf.nn.softmax_cross_entropy_with_logits(labels=lab, logits=v, name="xent")
        tf.nn.sparse_softmax_cross_entropy_with_logits(labels=ids, logits=v, name="sxent")
    return g


FETCHES = ["bc", "d2s", "s2d", "s2b", "b2s", "l2", "xent", "sxent"]


def feeds():
    x = rng.standard_normal((5, 4, 6, 8)).astype(np.float32)
    v = rng.standard_normal((5, 3)).astype(np.float32)
    lab = rng.dirichlet([1, 1, 1], 5).astype(np.float32)
    ids = rng.integers(0, 3, 5).astype(np.int32)
    return {"x": x, "v": v, "lab": lab, "ids": ids}


def test_more_ops_cpu():
    f = feeds()
    bc, d2s, s2d, s2b, b2s, l2, xent, sxent = run(graph_more(), FETCHES, f)
    x, v = f["x"], f["v"]
    np.testing.assert_array_equal(bc, np.broadcast_to(v[:, None, :], (5, 4, 3)))
    np.testing.assert_array_equal(d2s, d2s_ref(x, 2))
    np.testing.assert_array_equal(s2d, s2d_ref(x, 2))
    np.testing.assert_array_equal(d2s_ref(s2d, 2), x)
    np.testing.assert_array_equal(s2b, s2b_ref(x, [2, 3], [[1, 1], [0, 3]]))
    np.testing.assert_array_equal(b2s, x)  # BatchToSpaceND inverts SpaceToBatchND
    np.testing.assert_allclose(l2, (x.astype(np.float64) ** 2).sum() / 2, rtol=1e-5)
    lsm = torch.log_softmax(torch.as_tensor(v, dtype=torch.float64), 1).numpy()
    np.testing.assert_allclose(xent, -(f["lab"] * lsm).sum(1), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(sxent, -lsm[np.arange(5), f["ids"]], rtol=1e-5, atol=1e-6)


def test_atrous_conv2d_matches_dilated_conv():
    x = rng.standard_normal((2, 9, 11, 3))
    w = rng.standard_normal((3, 3, 3, 4))
    for padding in ("SAME", "VALID"):
        g = tf.Graph()
        with g.as_default():
            xi = tf.placeholder(tf.float64, [None, 9, 11, 3], name="x")
            tf.identity(tf.nn.atrous_conv2d(xi, tf.constant(w), 2, padding), name="a")
            tf.nn.conv2d(xi, tf.constant(w), [1, 1, 1, 1], padding, dilations=[1, 2, 2, 1], name="d")
        ops = {n.op for n in g.as_graph_def().node}
        assert {"SpaceToBatchND", "BatchToSpaceND"} <= ops
        a, d = run(g, ["a", "d"], {"x": x})
        assert a.shape == d.shape
        np.testing.assert_allclose(a, d, rtol=1e-10, atol=1e-10)


def test_softmax_xent_rows_are_separable():
    """One loss row per input row: the program may chunk a partition."""
    g = graph_more()
    prog = engine.program(g.serialize(), ["xent", "sxent"], ["v", "lab", "ids"])
    hints = {"v": (1, [7, 3]), "lab": (1, [7, 3]), "ids": (3, [7])}
    assert prog.row_separable(hints)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_more_ops_gpu_matches_cpu():
    f = feeds()
    g = graph_more()
    cpu = run(g, FETCHES, f)
    gpu = run(g, FETCHES, f, torch.device("cuda", 0))
    for name, a, b in zip(FETCHES, gpu, cpu):
        assert a.shape == b.shape, name
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5, err_msg=name)


def conv2d_transpose_ref(dy, w, out_shape, s, padding):
    """Direct definition: dx[n, h, w, ic] = sum dy[n, oh, ow, oc] * W[kh, kw, ic, oc]
    over h = oh*s + kh - pad_top (the forward conv's window positions)."""
    n, H, W, ic = out_shape
    kh, kw, _, oc = w.shape
    oh_, ow_ = dy.shape[1:3]
    if padding == "SAME":
        pt = max((oh_ - 1) * s + kh - H, 0) // 2
        pl = max((ow_ - 1) * s + kw - W, 0) // 2
    else:
        pt = pl = 0
    dx = np.zeros(out_shape)
    for oh in range(oh_):
        for ow in range(ow_):
            for a in range(kh):
                for b in range(kw):
                    h, x = oh * s + a - pt, ow * s + b - pl
                    if 0 <= h < H and 0 <= x < W:
                        dx[:, h, x, :] += dy[:, oh, ow, :] @ w[a, b].T
    return dx


@pytest.mark.parametrize("H,W,k,s,padding", [(8, 8, 3, 2, "SAME"), (7, 9, 3, 2, "SAME"), (6, 6, 3, 2, "VALID"),
                                             (5, 5, 2, 1, "SAME"), (9, 8, 4, 3, "VALID")])
def test_conv2d_transpose(H, W, k, s, padding):
    ic, oc, n = 3, 5, 2
    oh = -(-H // s) if padding == "SAME" else (H - k) // s + 1
    ow = -(-W // s) if padding == "SAME" else (W - k) // s + 1
    dy = rng.standard_normal((n, oh, ow, oc))
    w = rng.standard_normal((k, k, ic, oc))
    g = tf.Graph()
    with g.as_default():
        d = tf.placeholder(tf.float64, [None, oh, ow, oc], name="dy")
        tf.nn.conv2d_transpose(d, tf.constant(w), [n, H, W, ic], [1, s, s, 1], padding, name="dx")
    (dx,) = run(g, ["dx"], {"dy": dy})
    np.testing.assert_allclose(dx, conv2d_transpose_ref(dy, w, (n, H, W, ic), s, padding), rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("H,W,k,s,padding", [(8, 8, 3, 2, "SAME"), (7, 9, 3, 2, "SAME"), (6, 6, 3, 2, "VALID"),
                                             (16, 16, 4, 2, "SAME")])
def test_conv2d_transpose_gpu(H, W, k, s, padding):
    ic, oc, n = 8, 12, 3
    oh = -(-H // s) if padding == "SAME" else (H - k) // s + 1
    ow = -(-W // s) if padding == "SAME" else (W - k) // s + 1
    dy = rng.standard_normal((n, oh, ow, oc)).astype(np.float32)
    w = rng.standard_normal((k, k, ic, oc)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        d = tf.placeholder(tf.float32, [None, oh, ow, oc], name="dy")
        tf.nn.conv2d_transpose(d, tf.constant(w), [n, H, W, ic], [1, s, s, 1], padding, name="dx")
    (got,) = run(g, ["dx"], {"dy": dy}, torch.device("cuda", 0))
    want = conv2d_transpose_ref(dy.astype(np.float64), w.astype(np.float64), (n, H, W, ic), s, padding)
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)

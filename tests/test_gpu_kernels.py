"""Numerics of the HIP kernels: every op family executed by the native executor
on the GPU is compared against a plain PyTorch fp64/fp32 reference of the same
op on the host. Also checks that the device path really ran (the executor has
no silent ATen fallback on device tensors)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402

DEV = torch.device("cuda", 0)
rng = np.random.default_rng(1234)


def run(g, fetches, feeds, device=DEV):
    names = list(feeds)
    prog = engine.program(g.serialize(), fetches, names)
    ins = [torch.as_tensor(np.asarray(feeds[n])) for n in names]
    outs = engine.run_program(prog, ins, device)
    return [o.cpu() for o in outs]


def both(g, fetches, feeds):
    gpu = run(g, fetches, feeds, DEV)
    cpu = run(g, fetches, feeds, torch.device("cpu"))
    return gpu, cpu


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64])
@pytest.mark.parametrize("op", ["add", "subtract", "multiply", "maximum", "minimum", "div"])
def test_binary_same_and_broadcast(op, dtype):
    g = tf.Graph()
    with g.as_default():
        a = tf.placeholder(dtype, [None, 37], name="a")
        b = tf.placeholder(dtype, [None, 37], name="b")
        r = tf.placeholder(dtype, [37], name="r")
        s = tf.placeholder(dtype, [], name="s")
        f = getattr(tf, op)
        f(a, b, name="same")
        f(a, r, name="row")
        f(a, s, name="scal")
        f(s, a, name="lscal")
        f(tf.reshape(r, [37, 1]), tf.reshape(r, [1, 37]), name="bc")
    a_ = rng.integers(1, 9, (1001, 37)).astype(dtype)
    b_ = rng.integers(1, 9, (1001, 37)).astype(dtype)
    r_ = rng.integers(1, 9, (37,)).astype(dtype)
    s_ = np.asarray(3, dtype=dtype)
    gpu, cpu = both(g, ["same", "row", "scal", "lscal", "bc"], {"a": a_, "b": b_, "r": r_, "s": s_})
    for x, y in zip(gpu, cpu):
        assert x.shape == y.shape
        torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("op", ["sqrt", "exp", "log", "tanh", "sigmoid", "square", "negative", "abs",
                                "reciprocal", "floor", "ceil", "round", "sign", "sin", "cos"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_unary(op, dtype):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(dtype, [None], name="x")
        getattr(tf, op)(x, name="y")
    x_ = (rng.random(10007) * 3 + 0.1).astype(dtype)
    gpu, cpu = both(g, ["y"], {"x": x_})
    torch.testing.assert_close(gpu[0], cpu[0], rtol=2e-6 if dtype == np.float32 else 1e-12, atol=1e-6)


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64])
@pytest.mark.parametrize("red", ["reduce_sum", "reduce_min", "reduce_max", "reduce_mean"])
@pytest.mark.parametrize("shape,axes", [((4096, 33), [0]), ((33, 4096), [1]), ((7, 100003), [1]),
                                        ((300000, 8), [0]), ((6, 5, 4), [0, 2]), ((20, 30), [0, 1])])
def test_reductions(red, dtype, shape, axes):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(dtype, [None] * len(shape), name="x")
        getattr(tf, red)(x, axes, name="y")
    x_ = rng.integers(-50, 50, shape).astype(dtype)
    gpu, cpu = both(g, ["y"], {"x": x_})
    ref = torch.as_tensor(x_).double()
    if red == "reduce_sum":
        want = ref.sum(axes)
    elif red == "reduce_min":
        want = ref.amin(axes)
    elif red == "reduce_max":
        want = ref.amax(axes)
    else:
        want = cpu[0].double()  # integer mean truncation semantics come from the host path
        if np.issubdtype(dtype, np.floating):
            want = ref.mean(axes)
    torch.testing.assert_close(gpu[0].double(), want, rtol=1e-6, atol=1e-3)


def test_argminmax_softmax_topk():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 1000], name="x")
        tf.argmin(x, 1, name="amin")
        tf.argmax(x, 0, name="amax")
        tf.nn.softmax(x, name="sm")
        tf.nn.log_softmax(x, name="lsm")
        v, i = tf.nn.top_k(x, 5, name="top")
        tf.identity(v, name="tv")
        tf.identity(i, name="ti")
    x_ = rng.standard_normal((513, 1000)).astype(np.float32)
    gpu, cpu = both(g, ["amin", "amax", "sm", "lsm", "tv", "ti"], {"x": x_})
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_unsorted_segment_sum_and_gather():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, 100], name="x")
        ids = tf.placeholder(tf.int32, [None], name="ids")
        tf.unsorted_segment_sum(x, ids, 10, name="s")
        tf.unsorted_segment_max(x, ids, 12, name="m")
        tf.gather(x, ids, name="gth")
    x_ = rng.standard_normal((50000, 100))
    ids_ = rng.integers(0, 10, 50000).astype(np.int32)
    gpu, cpu = both(g, ["s", "m", "gth"], {"x": x_, "ids": ids_})
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("nseg", [10, 16, 37])
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
@pytest.mark.parametrize("n", [1, 777, 25000, 262144])
def test_small_int_segment_reduce_single_block(dtype, n, nseg):
    """The small integer paths (inner == 1, integer data, n <= 256k: register
    histograms in 1024-row blocks + a one-wave fold for <= 16 segments, one
    block of LDS atomics above):
    negative and out-of-range ids are dropped, empty segments of Min/Max get
    the type's extreme value, Sum of int32 wraps like the slab path."""
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(dtype, [None], name="x")
        ids = tf.placeholder(tf.int64, [None], name="ids")
        tf.unsorted_segment_sum(x, ids, nseg, name="s")
        tf.unsorted_segment_min(x, ids, nseg, name="lo")
        tf.unsorted_segment_max(x, ids, nseg, name="hi")
    x_ = rng.integers(-1000, 1000, n).astype(dtype)
    ids_ = rng.integers(-2, nseg + 3, n).astype(np.int64)  # some out of range; the top segments may stay empty
    gpu, cpu = both(g, ["s", "lo", "hi"], {"x": x_, "ids": ids_})
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32])
@pytest.mark.parametrize("shape", [(25000,), (3, 40000), (64, 1000), (5000,)])
def test_short_row_full_reduce_single_block(dtype, shape):
    """Rows that fit the one-block-per-row path (<= 256 KB, <= 64 rows)."""
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(dtype, [None] * len(shape), name="x")
        ax = len(shape) - 1
        tf.reduce_sum(x, [ax], name="s")
        tf.reduce_max(x, [ax], name="mx")
        tf.reduce_mean(x, [ax], name="mean")
    x_ = (rng.standard_normal(shape) * 100).astype(dtype)
    gpu, cpu = both(g, ["s", "mx", "mean"], {"x": x_})
    tol = 1e-5 if dtype == np.float32 else 1e-12
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b, rtol=tol, atol=tol * 100)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("m,n,k", [(1000, 512, 512), (129, 77, 33), (4096, 10, 100), (64, 128, 1000)])
def test_matmul_f32_mfma(m, n, k, ta, tb):
    g = tf.Graph()
    with g.as_default():
        a = tf.placeholder(tf.float32, None, name="a")
        b = tf.placeholder(tf.float32, None, name="b")
        tf.matmul(a, b, transpose_a=ta, transpose_b=tb, name="c")
    a_ = rng.uniform(-1, 1, (k, m) if ta else (m, k)).astype(np.float32)
    b_ = rng.uniform(-1, 1, (n, k) if tb else (k, n)).astype(np.float32)
    got = run(g, ["c"], {"a": a_, "b": b_})[0].double()
    A = torch.as_tensor(a_).double()
    B = torch.as_tensor(b_).double()
    want = (A.T if ta else A) @ (B.T if tb else B)
    # exact-f32 MFMA: error ~1e-7 * sum|a*b|
    tol = 4e-7 * k
    assert (got - want).abs().max().item() < tol


# one shape per f32 tile config / split-K path of csrc/kernels/gemm.hip plan_f32
@pytest.mark.parametrize("m,n,k,bias", [
    (300, 32, 2048, True),     # 128x32 tile + split-K with bias+relu in the reducer
    (5000, 64, 64, False),     # 128x64 -> 64x64 (too few blocks)
    (200, 200, 4096, True),    # 64x128 + 16-way split-K
    (70000, 100, 48, True),    # 128x128, ragged N
    (33, 1000, 999, False),    # odd K with split-K (scalar loads)
])
def test_matmul_f32_tiles_splitk(m, n, k, bias):
    g = tf.Graph()
    a_ = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    b_ = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    c_ = rng.uniform(-1, 1, n).astype(np.float32)
    with g.as_default():
        a = tf.placeholder(tf.float32, [None, k], name="a")
        y = tf.matmul(a, tf.constant(b_))
        if bias:
            y = tf.nn.relu(tf.nn.bias_add(y, tf.constant(c_)))
        tf.identity(y, name="c")
    got = run(g, ["c"], {"a": a_})[0].double()
    want = torch.as_tensor(a_).double() @ torch.as_tensor(b_).double()
    if bias:
        want = torch.clamp_min(want + torch.as_tensor(c_).double(), 0)
    assert (got - want).abs().max().item() < 4e-7 * k + 1e-6


def test_batch_matmul_splitk():
    g = tf.Graph()
    with g.as_default():
        a = tf.placeholder(tf.float32, [None, 100, 1024], name="a")
        b = tf.placeholder(tf.float32, [None, 1024, 70], name="b")
        tf.matmul(a, b, name="c")
    a_ = rng.uniform(-1, 1, (4, 100, 1024)).astype(np.float32)
    b_ = rng.uniform(-1, 1, (4, 1024, 70)).astype(np.float32)
    got = run(g, ["c"], {"a": a_, "b": b_})[0].double()
    want = torch.as_tensor(a_).double() @ torch.as_tensor(b_).double()
    assert (got - want).abs().max().item() < 4e-7 * 1024


@pytest.mark.parametrize("m,n,k", [(1000, 512, 512), (129, 77, 33), (100000, 10, 100)])
def test_matmul_f64_mfma(m, n, k):
    g = tf.Graph()
    with g.as_default():
        a = tf.placeholder(tf.float64, None, name="a")
        b = tf.placeholder(tf.float64, None, name="b")
        tf.matmul(a, b, transpose_b=True, name="c")
    a_ = rng.uniform(-1, 1, (m, k))
    b_ = rng.uniform(-1, 1, (n, k))
    got = run(g, ["c"], {"a": a_, "b": b_})[0]
    want = torch.as_tensor(a_) @ torch.as_tensor(b_).T
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-11)


def test_fused_gemm_bias_relu_identity_asymmetric():
    """A = I with an asymmetric B catches a row/col swapped C write."""
    g = tf.Graph()
    w = np.arange(512 * 512, dtype=np.float32).reshape(512, 512) / 1000.0
    bias = np.linspace(-300, 300, 512).astype(np.float32)
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 512], name="x")
        tf.nn.relu(tf.nn.bias_add(tf.matmul(x, tf.constant(w)), tf.constant(bias)), name="y")
    x_ = np.eye(512, dtype=np.float32)
    got = run(g, ["y"], {"x": x_})[0].numpy()
    want = np.maximum(w + bias, 0)
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-4)
    prog = engine.program(g.serialize(), ["y"], ["x"])
    assert "+bias +relu" in prog.describe([torch.as_tensor(x_).to(DEV)])


@pytest.mark.parametrize("cfg", [
    # (N, H, W, C, KH, KW, OC, stride, padding)
    (2, 17, 19, 3, 3, 3, 32, 2, "VALID"),
    (2, 35, 35, 64, 1, 1, 48, 1, "SAME"),
    (1, 17, 17, 128, 1, 7, 64, 1, "SAME"),
    (3, 8, 8, 32, 3, 3, 16, 1, "SAME"),
    (2, 9, 9, 20, 5, 5, 12, 2, "SAME"),
    (1, 8, 8, 256, 3, 3, 384, 1, "SAME"),   # small M, deep K: split-K conv
    (2, 13, 11, 20, 1, 1, 50, 1, "SAME"),   # pointwise conv, C % 4 != 0 (scalar GEMM path)
    (4, 35, 35, 192, 1, 1, 64, 1, "VALID"),  # pointwise conv -> plain GEMM, 128x64 tile
])
def test_conv2d_implicit_gemm(cfg):
    n, h, w_, c, kh, kw, oc, s, pad = cfg
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, h, w_, c], name="x")
        f = tf.placeholder(tf.float32, [kh, kw, c, oc], name="f")
        b = tf.placeholder(tf.float32, [oc], name="b")
        y = tf.nn.conv2d(x, f, [1, s, s, 1], pad, name="conv")
        tf.nn.relu(tf.nn.bias_add(y, b), name="y")
        tf.nn.max_pool(x, [1, 3, 3, 1], [1, 2, 2, 1], "SAME", name="mp")
        tf.nn.avg_pool(x, [1, 3, 3, 1], [1, 1, 1, 1], "SAME", name="ap")
    x_ = rng.standard_normal((n, h, w_, c)).astype(np.float32)
    f_ = rng.standard_normal((kh, kw, c, oc)).astype(np.float32) * 0.1
    b_ = rng.standard_normal(oc).astype(np.float32)
    gpu, cpu = both(g, ["y", "mp", "ap"], {"x": x_, "f": f_, "b": b_})
    for a, bb in zip(gpu, cpu):
        torch.testing.assert_close(a, bb, rtol=1e-4, atol=1e-4)


def test_data_movement_ops():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 6, 5], name="x")
        tf.transpose(x, [2, 0, 1], name="t")
        tf.concat([x, x * 2.0], 1, name="c")
        tf.tile(x, [2, 1, 3], name="ti")
        tf.identity(x[:, 1:5:2, ::-1], name="ss")
        tf.reshape(x, [-1, 30], name="rs")
        tf.stack([x, x], axis=1, name="st")
        tf.cast(x, tf.int32, name="ca")
        tf.one_hot(tf.cast(x[:, 0, 0], tf.int32), 4, name="oh")
        tf.where(x > 0.0, x, -x, name="w")
    x_ = rng.standard_normal((7, 6, 5)).astype(np.float32) * 3
    gpu, cpu = both(g, ["t", "c", "ti", "ss", "rs", "st", "ca", "oh", "w"], {"x": x_})
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b)


def test_native_extension_loaded():
    import sys
    mods = [m for m in sys.modules if m.endswith("tensorframes_amd._C")]
    assert mods, "native extension not loaded"


@pytest.mark.parametrize("align,half", [(False, False), (True, False), (False, True)])
@pytest.mark.parametrize("dtype", [np.uint8, np.float32])
def test_resize_bilinear_nearest(align, half, dtype):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.as_dtype(dtype), [None, 37, 29, 3], name="x")
        tf.image.resize_bilinear(x, [224, 224], align_corners=align, half_pixel_centers=half, name="bl")
        tf.image.resize_nearest_neighbor(x, [15, 64], align_corners=align, half_pixel_centers=half, name="nn")
    x_ = (rng.random((3, 37, 29, 3)) * 255).astype(dtype)
    gpu, cpu = both(g, ["bl", "nn"], {"x": x_})
    torch.testing.assert_close(gpu[0], cpu[0], rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(gpu[1], cpu[1], rtol=0, atol=0)


def test_cast_float_to_uint8_truncates():
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None], name="x")
        tf.cast(x, tf.uint8, name="u")
        tf.cast(x, tf.bool, name="b")
    x_ = np.array([0.0, 1.7, 200.2, 3.0], np.float32)
    gpu, cpu = both(g, ["u", "b"], {"x": x_})
    assert gpu[0].tolist() == [0, 1, 200, 3]
    assert gpu[1].tolist() == [False, True, True, True]
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a, b)


def test_extra_ops_gpu_vs_cpu():
    """Pad/MirrorPad, Split(V), Cumsum/Cumprod (row-block scan incl. chunk
    carry, and the strided-line path), LeakyRelu, ClipByValue, ReverseV2,
    DepthwiseConv2dNative, LRN, GatherNd: HIP kernels vs the CPU executor."""
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 700], name="x")
        img = tf.placeholder(tf.float32, [None, 13, 11, 8], name="img")
        ii = tf.placeholder(tf.int64, [None, 700], name="ii")
        tf.pad(x, [[1, 2], [3, 0]], constant_values=-2.0, name="pad")
        tf.pad(img, [[0, 0], [2, 1], [1, 3], [0, 0]], mode="REFLECT", name="refl")
        tf.pad(img, [[0, 0], [1, 1], [3, 2], [0, 0]], mode="SYMMETRIC", name="sym")
        tf.identity(tf.split(x, [100, -1, 50], axis=1)[1], name="split")
        tf.cumsum(x, 1, name="cs")
        tf.cumsum(x, 1, exclusive=True, reverse=True, name="cser")
        tf.cumsum(ii, 1, name="csi")
        tf.cumprod(x * 0.001 + 1.0, 0, name="cp")
        tf.nn.leaky_relu(x, 0.3, name="lr")
        tf.clip_by_value(x, -0.25, 0.5, name="clip")
        tf.reverse(img, [1, 3], name="rev")
        w = np.random.default_rng(2).standard_normal((3, 3, 8, 2)).astype(np.float32)
        tf.identity(tf.nn.depthwise_conv2d(img, tf.constant(w), [1, 2, 2, 1], "SAME"), name="dw")
        tf.nn.lrn(img, depth_radius=2, bias=1.0, alpha=0.5, beta=0.75, name="lrn")
        tf.gather_nd(img, tf.constant(np.array([[0, 1, 2], [2, 12, 10], [1, 0, 0]], np.int32)), name="gnd")
    x_ = rng.standard_normal((37, 700)).astype(np.float32)
    img_ = rng.standard_normal((3, 13, 11, 8)).astype(np.float32)
    ii_ = rng.integers(-5, 5, (37, 700))
    names = ["pad", "refl", "sym", "split", "cs", "cser", "csi", "cp", "lr", "clip", "rev", "dw", "lrn", "gnd"]
    gpu, cpu = both(g, names, {"x": x_, "img": img_, "ii": ii_})
    for n, a, b in zip(names, gpu, cpu):
        assert a.shape == b.shape, n
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-4, msg=n)

"""GEMM / Conv2D epilogue activations: MatMul (+BiasAdd) followed by one of
Relu, Relu6, Sigmoid, Tanh, Elu, Selu, Softplus is planned as ONE step (the
activation runs in the GEMM's register epilogue, or in the split-K reducer)
and matches an fp64 reference of the unfused ops. Runs on the host executor
and (gpu-marked) on the MFMA kernels."""
import numpy as np
import pytest
import torch

from tensorframes_amd import engine, tf

ACTS = {
    "relu": (tf.nn.relu, lambda x: np.maximum(x, 0)),
    "relu6": (tf.nn.relu6, lambda x: np.clip(x, 0, 6)),
    "sigmoid": (tf.nn.sigmoid, lambda x: 1 / (1 + np.exp(-x))),
    "tanh": (tf.nn.tanh, np.tanh),
    "elu": (tf.nn.elu, lambda x: np.where(x > 0, x, np.expm1(x))),
    "selu": (tf.nn.selu, lambda x: 1.0507009873554805 * np.where(x > 0, x, 1.6732632423543772 * np.expm1(x))),
    "softplus": (tf.nn.softplus, lambda x: np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20))))),
}


@pytest.fixture(params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def dev(request):
    if request.param == "cuda" and not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device(request.param, 0) if request.param == "cuda" else torch.device("cpu")


@pytest.mark.parametrize("act", sorted(ACTS))
@pytest.mark.parametrize("dtype,m,n,k", [
    (np.float32, 3000, 96, 128),
    (np.float32, 300, 32, 2048),   # split-K: the activation runs in the reducer
    (np.float64, 2000, 64, 100),
])
def test_matmul_bias_act_fused(dev, act, dtype, m, n, k):
    rng = np.random.default_rng(5)
    fn, ref = ACTS[act]
    w = (rng.standard_normal((k, n)) / np.sqrt(k)).astype(dtype)
    b = rng.uniform(-2, 2, n).astype(dtype)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32 if dtype == np.float32 else tf.float64, [None, k], name="x")
        fn(tf.nn.bias_add(tf.matmul(x, tf.constant(w)), tf.constant(b)), name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    x_ = rng.uniform(-3, 3, (m, k)).astype(dtype)
    xin = torch.as_tensor(x_).to(dev)
    plan = prog.describe([xin], dev.type == "cuda")
    assert f"+bias +{act}" in plan and "1 fused epilogues" in plan, plan
    got = engine.run_program(prog, [xin], dev)[0].cpu().double().numpy()
    want = ref(x_.astype(np.float64) @ w.astype(np.float64) + b.astype(np.float64))
    tol = (4e-7 * 3 * k + 2e-6) if dtype == np.float32 else 1e-11
    np.testing.assert_allclose(got, want, rtol=tol, atol=tol)


@pytest.mark.parametrize("act", ["sigmoid", "tanh", "elu"])
def test_conv_bias_act_fused(dev, act):
    rng = np.random.default_rng(6)
    fn, ref = ACTS[act]
    w = (rng.standard_normal((3, 3, 16, 24)) * 0.1).astype(np.float32)
    b = rng.uniform(-1, 1, 24).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 12, 12, 16], name="x")
        fn(tf.nn.bias_add(tf.nn.conv2d(x, tf.constant(w), [1, 1, 1, 1], "SAME"), tf.constant(b)), name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    x_ = rng.uniform(-1, 1, (4, 12, 12, 16)).astype(np.float32)
    xin = torch.as_tensor(x_).to(dev)
    assert f"+bias +{act}" in prog.describe([xin], dev.type == "cuda")
    got = engine.run_program(prog, [xin], dev)[0].cpu().double()
    xt = torch.as_tensor(x_).double().permute(0, 3, 1, 2)
    wt = torch.as_tensor(w).double().permute(3, 2, 0, 1)
    conv = torch.nn.functional.conv2d(xt, wt, padding=1).permute(0, 2, 3, 1) + torch.as_tensor(b).double()
    want = torch.as_tensor(ref(conv.numpy()))
    torch.testing.assert_close(got, want, rtol=2e-5, atol=2e-5)


def _run(dev, g, fetch, feeds):
    names = list(feeds)
    prog = engine.program(g.serialize(), [fetch], names)
    ins = [torch.as_tensor(feeds[n]).to(dev) for n in names]
    plan = prog.describe(ins, dev.type == "cuda")
    return plan, engine.run_program(prog, ins, dev)[0].cpu().double().numpy()


@pytest.mark.parametrize("dtype,m,n,k", [(np.float32, 3000, 96, 128), (np.float32, 300, 32, 2048),
                                         (np.float64, 1000, 64, 100)])
def test_matmul_absorbs_elementwise_chain(dev, dtype, m, n, k):
    """relu(x@W + b) * 0.5 + c[N] - z[M,N] (z a feed) , then max with r[M,1]
    and a square: ONE GEMM step whose epilogue runs the whole chain."""
    rng = np.random.default_rng(7)
    tdt = tf.float32 if dtype == np.float32 else tf.float64
    w = (rng.standard_normal((k, n)) / np.sqrt(k)).astype(dtype)
    b, c = rng.uniform(-1, 1, n).astype(dtype), rng.uniform(-1, 1, n).astype(dtype)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tdt, [None, k], name="x")
        z = tf.placeholder(tdt, [None, n], name="z")
        r = tf.placeholder(tdt, [None, 1], name="r")
        h = tf.nn.relu(tf.nn.bias_add(tf.matmul(x, tf.constant(w)), tf.constant(b)))
        h = (h * 0.5 + tf.constant(c)) - z
        h = tf.maximum(h, r)
        tf.multiply(h, h, name="y")
    x_ = rng.uniform(-2, 2, (m, k)).astype(dtype)
    z_ = rng.uniform(-1, 1, (m, n)).astype(dtype)
    r_ = rng.uniform(-1, 1, (m, 1)).astype(dtype)
    plan, got = _run(dev, g, "y", {"x": x_, "z": z_, "r": r_})
    assert "+bias +relu +epi[mul:scalar,add:col,sub:full,max:row,square]" in plan, plan
    assert "plan: 1 steps" in plan, plan
    h = np.maximum(x_.astype(np.float64) @ w.astype(np.float64) + b, 0) * 0.5 + c - z_
    want = np.maximum(h, r_) ** 2
    tol = (4e-7 * 3 * k + 1e-5) if dtype == np.float32 else 1e-10
    np.testing.assert_allclose(got, want, rtol=tol, atol=tol)


def test_matmul_chain_reversed_operands_and_runtime_scalar(dev):
    """2 / (x@W) style reversed operands (rdiv, rsub) and a 1-element runtime
    tensor operand."""
    rng = np.random.default_rng(8)
    w = (rng.standard_normal((64, 48)) / 8).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 64], name="x")
        s = tf.placeholder(tf.float32, [], name="s")
        h = tf.matmul(x, tf.constant(w))
        h = 3.0 - tf.abs(h)                 # rsub:scalar after abs
        h = tf.constant(2.0, tf.float32) / h  # rdiv:scalar
        tf.multiply(s, tf.tanh(h), name="y")  # tanh, mul by runtime scalar
    x_ = rng.uniform(-0.2, 0.2, (500, 64)).astype(np.float32)
    plan, got = _run(dev, g, "y", {"x": x_, "s": np.float32(1.5)})
    assert "+epi[abs,rsub:scalar,rdiv:scalar,tanh,mul:scalar]" in plan, plan
    want = 1.5 * np.tanh(2.0 / (3.0 - np.abs(x_.astype(np.float64) @ w)))
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)


def test_batch_matmul_chain_full_and_col(dev):
    rng = np.random.default_rng(9)
    g = tf.Graph()
    c = rng.uniform(-1, 1, 24).astype(np.float32)
    with g.as_default():
        a = tf.placeholder(tf.float32, [None, 40, 32], name="a")
        bm = tf.placeholder(tf.float32, [None, 32, 24], name="b")
        z = tf.placeholder(tf.float32, [None, 40, 24], name="z")
        tf.add(tf.matmul(a, bm) * tf.constant(c), z, name="y")
    a_ = rng.uniform(-1, 1, (3, 40, 32)).astype(np.float32)
    b_ = rng.uniform(-1, 1, (3, 32, 24)).astype(np.float32)
    z_ = rng.uniform(-1, 1, (3, 40, 24)).astype(np.float32)
    plan, got = _run(dev, g, "y", {"a": a_, "b": b_, "z": z_})
    assert "+epi[mul:col,add:full]" in plan, plan
    want = (a_.astype(np.float64) @ b_.astype(np.float64)) * c + z_
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)


def test_conv_absorbs_chain(dev):
    rng = np.random.default_rng(10)
    w = (rng.standard_normal((3, 3, 8, 16)) * 0.1).astype(np.float32)
    b = rng.uniform(-1, 1, 16).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 10, 10, 8], name="x")
        z = tf.placeholder(tf.float32, [None, 10, 10, 16], name="z")
        h = tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(x, tf.constant(w), [1, 1, 1, 1], "SAME"), tf.constant(b)))
        tf.add(h * 2.0, z, name="y")  # residual add
    x_ = rng.uniform(-1, 1, (2, 10, 10, 8)).astype(np.float32)
    z_ = rng.uniform(-1, 1, (2, 10, 10, 16)).astype(np.float32)
    plan, got = _run(dev, g, "y", {"x": x_, "z": z_})
    assert "+bias +relu +epi[mul:scalar,add:full]" in plan, plan
    xt = torch.as_tensor(x_).double().permute(0, 3, 1, 2)
    wt = torch.as_tensor(w).double().permute(3, 2, 0, 1)
    conv = torch.nn.functional.conv2d(xt, wt, padding=1).permute(0, 2, 3, 1) + torch.as_tensor(b).double()
    want = torch.clamp_min(conv, 0).numpy() * 2.0 + z_
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)


def test_chain_stops_at_fetched_intermediate(dev):
    """An intermediate that is also fetched stays materialised: the chain ends there."""
    rng = np.random.default_rng(11)
    w = rng.standard_normal((16, 8)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 16], name="x")
        h = tf.multiply(tf.matmul(x, tf.constant(w)), 2.0, name="h")
        tf.add(h, 1.0, name="y")
    prog = engine.program(g.serialize(), ["h", "y"], ["x"])
    x_ = torch.as_tensor(rng.uniform(-1, 1, (64, 16)).astype(np.float32)).to(dev)
    plan = prog.describe([x_], dev.type == "cuda")
    assert "+epi[mul:scalar]" in plan and "add" not in plan.split("+epi[mul:scalar]")[1].split("\n")[0], plan
    h_, y_ = [o.cpu().numpy() for o in engine.run_program(prog, [x_], dev)]
    np.testing.assert_allclose(y_, h_ + 1.0, rtol=1e-6)


def test_chain_operand_produced_after_the_matmul(dev):
    """The chain's full-size operand is computed by a node that follows the
    MatMul in topological order: the fused step runs at the chain's last op."""
    rng = np.random.default_rng(12)
    w = rng.standard_normal((16, 8)).astype(np.float32)
    b = rng.standard_normal(8).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 16], name="x")
        x3 = tf.placeholder(tf.float32, [None, 8, 4], name="x3")
        h = tf.nn.bias_add(tf.matmul(x, tf.constant(w)), tf.constant(b))
        z = tf.reduce_sum(x3, [2])          # produced after the MatMul
        c = tf.reduce_max(x3, [1, 2])        # per-row [M] -> [M, 1]
        tf.subtract(h, z) * tf.reshape(c, [-1, 1])
        tf.identity(tf.subtract(h, z) * tf.reshape(c, [-1, 1]), name="y")
    x_ = rng.uniform(-1, 1, (64, 16)).astype(np.float32)
    x3_ = rng.uniform(-1, 1, (64, 8, 4)).astype(np.float32)
    plan, got = _run(dev, g, "y", {"x": x_, "x3": x3_})
    assert "+bias +epi[sub:full" in plan, plan
    want = (x_.astype(np.float64) @ w + b - x3_.sum(2)) * x3_.max((1, 2))[:, None]
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)


def test_matmul_chain_max_min_propagate_nan(dev):
    """An absorbed Maximum/Minimum propagates NaN from either side, exactly as
    the unfused elementwise kernels (and np.maximum / np.minimum) do."""
    rng = np.random.default_rng(9)
    w = (rng.standard_normal((32, 16)) / 6).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 32], name="x")
        r = tf.placeholder(tf.float32, [None, 1], name="r")
        z = tf.placeholder(tf.float32, [None, 16], name="z")
        tf.minimum(tf.maximum(tf.matmul(x, tf.constant(w)), r), z, name="y")
    x_ = rng.uniform(-1, 1, (300, 32)).astype(np.float32)
    r_ = rng.uniform(-1, 1, (300, 1)).astype(np.float32)
    z_ = rng.uniform(-1, 1, (300, 16)).astype(np.float32)
    x_[0, 3] = np.nan   # NaN accumulator
    r_[1, 0] = np.nan   # NaN max operand
    z_[2, 5] = np.nan   # NaN min operand
    plan, got = _run(dev, g, "y", {"x": x_, "r": r_, "z": z_})
    assert "+epi[max:row,min:full]" in plan, plan
    want = np.minimum(np.maximum(x_.astype(np.float64) @ w, r_), z_)
    assert np.isnan(got[0]).all() and np.isnan(got[1]).all() and np.isnan(got[2, 5])
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)

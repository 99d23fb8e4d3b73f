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

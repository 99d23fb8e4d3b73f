"""Planner-fused pools (GPU): MaxPool/AvgPool -> BiasAdd -> Relu/Relu6 run as
one pool kernel, and a pool whose only consumer is a last-axis ConcatV2 writes
its channel slice of the concat output in place. Checked against an fp64
numpy reference of the unfused graph (TF SAME/VALID pooling; avg over the
valid taps)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402

DEV = torch.device("cuda", 0)


def pool_ref(x, k, s, pad, is_max):
    n, h, w, c = x.shape
    if pad == "SAME":
        oh, ow = -(-h // s), -(-w // s)
        ph, pw = max((oh - 1) * s + k - h, 0), max((ow - 1) * s + k - w, 0)
        pt, pl = ph // 2, pw // 2
    else:
        oh, ow = (h - k) // s + 1, (w - k) // s + 1
        pt = pl = 0
    y = np.zeros((n, oh, ow, c))
    for i in range(oh):
        for j in range(ow):
            h0, w0 = i * s - pt, j * s - pl
            win = x[:, max(h0, 0):min(h0 + k, h), max(w0, 0):min(w0 + k, w)]
            y[:, i, j] = win.max(axis=(1, 2)) if is_max else win.mean(axis=(1, 2))
    return y


def run(g, fetch, x):
    prog = engine.program(g.serialize(), [fetch], ["x"])
    desc = prog.describe([torch.from_numpy(x)], as_gpu=True)
    out = engine.run_program(prog, [torch.from_numpy(x)], DEV)[0].cpu().numpy()
    return out, desc


@pytest.mark.parametrize("is_max,k,s,pad,c,act", [
    (False, 3, 1, "SAME", 32, "relu"),   # Inception pool branch
    (True, 3, 2, "VALID", 24, "relu6"),
    (False, 2, 2, "SAME", 7, None),      # odd channels: scalar path, bias only
])
def test_pool_bias_act_fused(is_max, k, s, pad, c, act):
    rng = np.random.default_rng(c + k)
    x = rng.uniform(-1, 1, (3, 11, 13, c)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, c).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, 11, 13, c], name="x")
        pool = tf.nn.max_pool if is_max else tf.nn.avg_pool
        y = tf.nn.bias_add(pool(xi, [1, k, k, 1], [1, s, s, 1], pad), tf.constant(b))
        y = {"relu": tf.nn.relu, "relu6": tf.nn.relu6, None: tf.identity}[act](y)
        tf.identity(y, name="y")
    got, desc = run(g, "y", x)
    want = pool_ref(x.astype(np.float64), k, s, pad, is_max) + b
    if act == "relu":
        want = np.maximum(want, 0)
    elif act == "relu6":
        want = np.clip(want, 0, 6)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
    assert "+bias" in desc


def test_pool_branch_written_into_concat_slice():
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, (4, 9, 9, 16)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, (1, 1, 16, 20)).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, 12).astype(np.float32)
    wp = rng.uniform(-0.3, 0.3, (1, 1, 16, 12)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, 9, 9, 16], name="x")
        a = tf.nn.relu(tf.nn.conv2d(xi, tf.constant(w), [1, 1, 1, 1], "SAME"))
        p = tf.nn.conv2d(xi, tf.constant(wp), [1, 1, 1, 1], "SAME")
        p = tf.nn.relu(tf.nn.bias_add(tf.nn.avg_pool(p, [1, 3, 3, 1], [1, 1, 1, 1], "SAME"), tf.constant(b)))
        m = tf.nn.max_pool(xi, [1, 3, 3, 1], [1, 1, 1, 1], "SAME")
        tf.concat([a, p, m], 3, name="y")
    got, desc = run(g, "y", x)
    x64 = x.astype(np.float64)
    want_a = np.maximum(x64 @ w[0, 0], 0)
    want_p = np.maximum(pool_ref(x64 @ wp[0, 0], 3, 1, "SAME", False) + b, 0)
    want_m = pool_ref(x64, 3, 1, "SAME", True)
    np.testing.assert_allclose(got, np.concatenate([want_a, want_p, want_m], 3), rtol=1e-5, atol=1e-5)
    assert "(3 inputs written in place)" in desc, desc


def test_nested_concat_written_in_place():
    """Inception-v3 Mixed_7b/7c: concat([b0, concat([b1a, b1b]), concat([b2a, b2b]), pool]);
    the inner concats' producers write straight into the outer concat."""
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, (2, 5, 5, 8)).astype(np.float32)
    ws = [rng.uniform(-0.3, 0.3, (1, 1, 8, oc)).astype(np.float32) for oc in (12, 8, 4, 16, 20)]
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.float32, [None, 5, 5, 8], name="x")
        cv = [tf.nn.relu(tf.nn.conv2d(xi, tf.constant(w), [1, 1, 1, 1], "SAME")) for w in ws]
        y1 = tf.nn.conv2d(cv[1], tf.constant(rng.uniform(-0.3, 0.3, (1, 3, 8, 8)).astype(np.float32)),
                          [1, 1, 1, 1], "SAME")
        inner1 = tf.concat([tf.nn.relu(y1), cv[2]], 3)
        inner2 = tf.concat([cv[3], cv[4]], 3)
        tf.concat([cv[0], inner1, inner2], 3, name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    desc = prog.describe([torch.from_numpy(x)], as_gpu=True)
    got = engine.run_program(prog, [torch.from_numpy(x)], DEV)[0].cpu().numpy()
    want = engine.run_program(prog, [torch.from_numpy(x)], torch.device("cpu"))[0].numpy()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
    assert desc.count("OP   ConcatV2") == 3
    assert "(3 inputs written in place)" in desc, desc

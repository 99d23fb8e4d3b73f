"""Horizontal fusion of sibling convs (GPU plans): Conv2Ds reading the same
input with the same geometry run as ONE implicit GEMM over their
concatenated filters, each member writing its own output or concat slice
(segmented epilogue, kernels/gemm.hip out_col). Checked against the host
executor's ATen fp32 convs (Inception mixed blocks)."""
import numpy as np
import pytest
import torch

from tensorframes_amd import engine, tf


def _graph(rng, ocs, k=1, act=tf.nn.relu, bias=True, cin=16, hw=12, concat_all=True, extra_branch=True):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, hw, hw, cin], name="x")

        def conv(inp, oc, kk, name):
            w = tf.constant((rng.standard_normal((kk, kk, int(inp.get_shape()[3]), oc)) * 0.2).astype(np.float32))
            y = tf.nn.conv2d(inp, w, [1, 1, 1, 1], "SAME")
            if bias:
                y = tf.nn.bias_add(y, tf.constant(rng.uniform(-1, 1, oc).astype(np.float32)))
            return act(y, name=name)
        heads = [conv(x, oc, k, f"h{i}") for i, oc in enumerate(ocs)]
        outs = list(heads)
        if extra_branch:  # one head feeds a further conv (not a concat slice)
            outs[1] = conv(heads[1], 8, 3, "tail")
        if concat_all:
            tf.concat(outs, 3, name="y")
        else:
            tf.identity(tf.add_n([tf.reduce_sum(o, [3], keep_dims=True) for o in outs]), name="y")
    return g


def _check(g, xin, dev, n_fused):
    prog = engine.program(g.serialize(), ["y"], ["x"])
    plan = prog.describe([xin], True)
    assert f"{n_fused} sibling convs fused" in plan, plan
    want = engine.run_program(prog, [xin], torch.device("cpu"))[0].double()
    got = engine.run_program(prog, [xin.to(dev)], dev)[0].cpu().double()
    torch.testing.assert_close(got, want, rtol=2e-5, atol=2e-5)
    return plan


def test_plan_describes_fused_siblings():
    g = _graph(np.random.default_rng(0), [24, 8, 12])
    prog = engine.program(g.serialize(), ["y"], ["x"])
    plan = prog.describe([torch.rand(2, 12, 12, 16)], True)
    assert "3 sibling convs fused" in plan and "siblings[" in plan, plan
    # the host plan keeps the convs separate (ATen reference path)
    assert "sibling" not in prog.describe([torch.rand(2, 12, 12, 16)], False)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
@pytest.mark.parametrize("bias", [True, False])
def test_sibling_convs_match_host(k, act, bias):
    dev = _gpu()
    rng = np.random.default_rng(1)
    fn = tf.nn.relu if act == "relu" else tf.nn.sigmoid
    g = _graph(rng, [24, 8, 12], k=k, act=fn, bias=bias)
    _check(g, torch.rand(3, 12, 12, 16), dev, 3)


@pytest.mark.gpu
def test_five_siblings_split_into_groups_of_four():
    dev = _gpu()
    g = _graph(np.random.default_rng(2), [16, 8, 20, 4, 12], concat_all=False)
    _check(g, torch.rand(2, 12, 12, 16), dev, 4)


@pytest.mark.gpu
def test_sibling_convs_split_k_reducer():
    # tiny M, deep K: the merged GEMM runs split-K and the reducer writes the segments
    dev = _gpu()
    g = _graph(np.random.default_rng(3), [32, 32, 48], cin=512, hw=4, extra_branch=False)
    _check(g, torch.rand(1, 4, 4, 512), dev, 3)


def _pool_branch_graph(rng, cin=16, hw=12):
    """An Inception mixed block: three 1x1 heads on x plus AvgPool -> 1x1 conv."""
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, hw, hw, cin], name="x")

        def conv(inp, oc, name):
            w = tf.constant((rng.standard_normal((1, 1, int(inp.get_shape()[3]), oc)) * 0.2).astype(np.float32))
            b = tf.constant(rng.uniform(-1, 1, oc).astype(np.float32))
            return tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(inp, w, [1, 1, 1, 1], "SAME"), b), name=name)
        heads = [conv(x, 24, "h0"), conv(x, 8, "h1"), conv(x, 12, "h2")]
        pooled = tf.nn.avg_pool(x, [1, 3, 3, 1], [1, 1, 1, 1], "SAME")
        tf.concat(heads + [conv(pooled, 16, "pool_proj")], 3, name="y")
    return g


def test_avgpool_then_pointwise_conv_is_reordered_and_value_preserving():
    import tensorframes_amd as tfs
    from tensorframes_amd.graph import rewrite
    g = _pool_branch_graph(np.random.default_rng(4))
    out = rewrite.optimize(g.serialize())
    assert out is not None
    xin = torch.rand(2, 12, 12, 16)
    engine.clear_program_cache()
    prog = engine.program(g.serialize(), ["y"], ["x"])
    plan = prog.describe([xin], True)
    # the pool branch's conv now reads x and joins the 1x1 siblings; the pool runs on its 16 channels
    assert "4 sibling convs fused" in plan, plan
    got = engine.run_program(prog, [xin], torch.device("cpu"))[0].double()
    tfs.set_config(graph_rewrites=False)
    try:
        engine.clear_program_cache()
        ref = engine.program(g.serialize(), ["y"], ["x"])
        assert "3 sibling convs fused" in ref.describe([xin], True)  # the pool branch stays apart
        want = engine.run_program(ref, [xin], torch.device("cpu"))[0].double()
    finally:
        tfs.set_config(graph_rewrites=True)
        engine.clear_program_cache()
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_pool_branch_fused_siblings_match_host():
    dev = _gpu()
    g = _pool_branch_graph(np.random.default_rng(5))
    _check(g, torch.rand(3, 12, 12, 16), dev, 4)

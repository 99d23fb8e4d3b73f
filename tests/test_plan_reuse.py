"""Plan reuse across rebuilt graphs: a graph that differs
from an earlier one only in the payloads of its parameter constants has the
same Graph::structure_key, and its program takes over the earlier program's
plans (Program::adopt) with the new constant values. Reference workload:
src/main/python/tensorframes_snippets/kmeans_demo.py:101-168 (the graphs are
rebuilt with new centres every iteration)."""
import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import engine, tf
from tensorframes_amd._native import _C
from tensorframes_amd.models import kmeans
from tensorframes_amd.utils.logging import metrics


def _graph(w, bias=None, scale=2.0):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, w.shape[0]], name="x")
        y = tf.matmul(x, tf.constant(w)) * scale
        if bias is not None:
            y = y + tf.constant(bias)
        tf.identity(tf.reduce_sum(tf.square(tf.constant(w)), 0) + y, name="y")
    return g.serialize()


def _devices():
    devs = ["cpu"]
    if torch.cuda.is_available():
        devs.append("cuda")
    return devs


def test_structure_key_ignores_parameter_payloads_only():
    rng = np.random.default_rng(0)
    w1, w2 = rng.standard_normal((5, 3)), rng.standard_normal((5, 3))
    k = lambda b: _C.Graph(b).structure_key()  # noqa: E731
    assert k(_graph(w1)) == k(_graph(w2))
    assert k(_graph(w1)) != k(_graph(w1[:, :2].copy()))  # a shape is structure
    assert k(_graph(w1, scale=2.0)) != k(_graph(w1, scale=3.0))  # a scalar is baked: structure
    assert k(_graph(w1, bias=np.ones(3))) == k(_graph(w1, bias=np.zeros(3)))
    g = _C.Graph(_graph(w1, bias=np.ones(3)))
    assert sorted(g.parameter_consts()) == ["Const", "Const_1", "Const_2"]


def test_integer_or_scalar_derived_constants_are_not_parameters():
    # a float constant whose folded value becomes a shape (via Cast) or a
    # scalar must stay part of the structure
    def gb(v):
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float64, [None], name="x")
            c = tf.constant(np.asarray(v, np.float64))
            n = tf.cast(tf.reduce_sum(c), tf.int32)
            tf.identity(x * tf.cast(n, tf.float64), name="y")
        return g.serialize()
    k = lambda b: _C.Graph(b).structure_key()  # noqa: E731
    assert k(gb([1.0, 2.0])) != k(gb([1.0, 3.0]))
    assert _C.Graph(gb([1.0, 2.0])).parameter_consts() == []


@pytest.mark.parametrize("dev", _devices())
def test_adopted_program_uses_new_values_and_old_one_keeps_its_own(dev):
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((64, 5))).to(dev)
    ws = [rng.standard_normal((5, 3)) for _ in range(4)]
    bs = [rng.standard_normal(3) for _ in range(4)]
    engine.clear_program_cache()
    metrics.reset()
    progs = []
    for w, b in zip(ws, bs):
        p = engine.program(_graph(w, b), ["y"], ["x"])
        for _ in range(5):  # enough runs for a HIP-graph capture on the GPU
            out = engine.run_program(p, [x], torch.device(dev))[0]
        ref = (x.cpu().double() @ torch.from_numpy(w)) * 2.0 + torch.from_numpy(b) + \
            torch.from_numpy((w ** 2).sum(0))
        assert torch.allclose(out.cpu().double(), ref, rtol=1e-10, atol=1e-10)
        progs.append(p)
    assert metrics.snapshot().get("programs_adopted", 0) == 3
    st = progs[-1].stats()
    assert st["plans_adopted"] >= 1 and st["plans_built"] == 0
    # the first program (its plans were taken over) still computes with ITS constants
    out0 = engine.run_program(progs[0], [x], torch.device(dev))[0]
    ref0 = (x.cpu().double() @ torch.from_numpy(ws[0])) * 2.0 + torch.from_numpy(bs[0]) + \
        torch.from_numpy((ws[0] ** 2).sum(0))
    assert torch.allclose(out0.cpu().double(), ref0, rtol=1e-10, atol=1e-10)
    assert progs[0].stats()["plans_built"] >= 1


def test_kmeans_iterations_adopt_plans_and_match_numpy():
    rng = np.random.default_rng(3)
    pts = rng.uniform(0.0, 1.0, size=(2000, 8))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4)).cache()
    c = pts[rng.choice(2000, 5, replace=False)].copy()  # every centre owns points
    engine.clear_program_cache()
    metrics.reset()
    for _ in range(4):
        c1, d1 = kmeans.run_one_step2(df, c)
        ref, dref = kmeans.numpy_step(pts, c)
        np.testing.assert_allclose(c1, ref, rtol=1e-6, atol=1e-9)
        assert abs(d1 - dref) <= 1e-9 * abs(dref)
        c = c1
    snap = metrics.snapshot()
    assert snap.get("programs_adopted", 0) + snap.get("programs_rebound", 0) >= 3


def test_plan_reuse_can_be_disabled():
    rng = np.random.default_rng(4)
    engine.clear_program_cache()
    metrics.reset()
    tfs.set_config(plan_reuse=False)
    try:
        for _ in range(3):
            engine.program(_graph(rng.standard_normal((5, 3))), ["y"], ["x"])
    finally:
        tfs.set_config(plan_reuse=True)
    assert metrics.snapshot().get("programs_adopted", 0) == 0


def _spec_graph(w, ints, name_suffix=""):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, w.shape[0]], name="x")
        y = tf.matmul(x, tf.constant(w))
        y = tf.tile(y, tf.constant(ints))  # an integer constant: structure, never a parameter
        tf.identity(y * 0.5, name="y")
    return g


@pytest.mark.parametrize("device", _devices())
def test_program_for_spec_rebinds_parameters_and_checks_the_rest(device):
    """DSL graphs rebuilt with new float payloads get the known program with
    the payloads swapped (Program.rebind, no serialise/parse); a change in an
    integer constant is a different structure and must not reuse it."""
    from tensorframes_amd import core
    engine.clear_program_cache()
    rng = np.random.default_rng(5)
    x = rng.standard_normal((64, 4))
    dev = torch.device(device)
    before = metrics.snapshot().get("programs_rebound", 0)
    for it in range(4):
        w = rng.standard_normal((4, 3))
        ints = [1, 2] if it < 3 else [2, 1]
        g = _spec_graph(w, ints)
        spec = core._resolve([g.get_tensor_by_name("y:0")])
        prog = engine.program_for_spec(spec, ["y:0"], ["x"])
        got = engine.run_program(prog, [torch.as_tensor(x)], dev)[0].cpu().numpy()
        want = np.tile(x @ w, ints) * 0.5
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    # iterations 1 and 2 rebind; iteration 3 changed the int constant: a new program
    assert metrics.snapshot().get("programs_rebound", 0) - before == 2


def test_rebind_refuses_non_parameters():
    rng = np.random.default_rng(6)
    g = _spec_graph(rng.standard_normal((4, 3)), [1, 2])
    prog = engine.program(g.serialize(), ["y:0"], ["x"])
    with pytest.raises(Exception, match="not a parameter constant"):
        prog.rebind({"x": torch.zeros(4, 3, dtype=torch.float64)})
    with pytest.raises(Exception, match="values of its dtype"):
        prog.rebind({"Const": torch.zeros(5, 3, dtype=torch.float64)})

"""Planner fusion: elementwise regions and row reductions with fused
prologues become ONE generated kernel (runtime/fusion.cpp, JIT-compiled by
hiprtc for gfx950). CPU tests check the plan and compile the generated
sources; GPU tests compare fused results against the per-op CPU oracle.

Reference workload: the K-Means distance graph
(src/main/python/tensorframes_snippets/kmeans_demo.py:31-42)."""
import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import engine, tf
from tensorframes_amd._native import _C


def _kmeans_graph(k=10, f=100):
    from tensorframes_amd.models.kmeans import tf_compute_distances
    c = np.random.default_rng(0).standard_normal((k, f))
    g = tf.Graph()
    with g.as_default():
        points = tf.placeholder(tf.double, shape=[None, f], name="features")
        distances = tf_compute_distances(points, c)
        tf.argmin(distances, 1, name="indexes")
        tf.reduce_min(distances, 1, name="min_distances")
        tf.identity(distances, name="d")
    return g.serialize(), c


def test_kmeans_distance_chain_is_one_kernel():
    gb, _ = _kmeans_graph()
    prog = engine.program(gb, ["indexes", "min_distances"], ["features"])
    x = [torch.zeros(25000, 100, dtype=torch.float64)]
    plan = prog.describe(x, True)
    # 2 * prods runs in the GEMM epilogue; t1 + t2 - (2 * prods) (two Tiles,
    # ExpandDims, Add, Sub) is evaluated inside the ArgMin/Min row reduction;
    # Square -> Sum as one row reduction
    assert "FUSED-ROWRED indexes [Tile ExpandDims Tile Add Sub -> ArgMin Min]" in plan, plan
    assert "FUSED-ROWRED distances/Sum [Square -> Sum]" in plan, plan
    assert "GEMM MatMul distances/MatMul -> distances/mul +epi[mul:scalar]" in plan, plan
    assert plan.startswith("plan: 3 steps"), plan  # was 9 unfused kernels
    # the host plan is unfused (ATen oracle path)
    assert "FUSED" not in prog.describe(x)


def test_distance_chain_fetched_is_an_elementwise_region():
    gb, _ = _kmeans_graph()
    prog = engine.program(gb, ["d"], ["features"])
    plan = prog.describe([torch.zeros(1000, 100, dtype=torch.float64)], True)
    # t1 = tile(center_squares, [rows, 1]) depends on the fed shape: it is not
    # folded into a row-sized host constant (graph.cpp kDynFoldLimit) but read
    # inside the region
    assert "FUSED d [Tile ExpandDims Tile Add Sub Identity]" in plan, plan
    small = prog.describe([torch.zeros(40, 100, dtype=torch.float64)], True)
    assert "FUSED d [ExpandDims Tile Add Sub Identity]" in small, small  # 40x10: folded


def test_generated_sources_compile_for_gfx950():
    gb, _ = _kmeans_graph()
    prog = engine.program(gb, ["indexes", "min_distances", "d"], ["features"])
    srcs = prog.fused_sources([torch.zeros(5000, 100, dtype=torch.float64)])
    assert len(srcs) >= 2
    for s in srcs:
        assert _C.jit_compile(s) > 1000  # a code object


def _ew_graph(dt):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(dt, [None, 7, 5], name="x")
        b = tf.placeholder(dt, [5], name="b")
        c = tf.constant(np.arange(7, dtype=dt.as_numpy_dtype).reshape(7, 1) + 1)
        y = tf.maximum(x * b + c, tf.cast(tf.constant(2), dt)) - tf.square(b)
        if dt in (tf.float32, tf.float64):
            y = tf.nn.relu(tf.exp(y * 0.01)) / (c + 1.0)
        tf.identity(y, name="y")
    return g.serialize()


@pytest.mark.parametrize("dt", [tf.float32, tf.float64, tf.int32, tf.int64])
def test_elementwise_region_plan(dt):
    prog = engine.program(_ew_graph(dt), ["y"], ["x", "b"])
    npdt = dt.as_numpy_dtype
    ins = [torch.zeros(300, 7, 5, dtype=torch.from_numpy(np.zeros(1, npdt)).dtype),
           torch.zeros(5, dtype=torch.from_numpy(np.zeros(1, npdt)).dtype)]
    plan = prog.describe(ins, True)
    assert "fused regions" in plan and "FUSED" in plan, plan
    for s in prog.fused_sources(ins):
        assert _C.jit_compile(s) > 0


def test_fusion_can_be_disabled_per_process(monkeypatch):
    import subprocess
    import sys
    code = ("import torch, numpy as np; import tensorframes_amd as tfs; from tensorframes_amd import engine, tf\n"
            "from tests.test_fusion import _kmeans_graph\n"
            "gb, _ = _kmeans_graph(); p = engine.program(gb, ['indexes'], ['features'])\n"
            "print(p.describe([torch.zeros(1000, 100, dtype=torch.float64)], True))\n")
    import os
    env = dict(os.environ, TFA_FUSION="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert "0 fused regions" in out.stdout


# ---------------------------------------------------------------- GPU numerics
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [tf.float32, tf.float64, tf.int32, tf.int64])
def test_elementwise_region_matches_oracle_gpu(dt):
    dev = _gpu()
    prog = engine.program(_ew_graph(dt), ["y"], ["x", "b"])
    npdt = dt.as_numpy_dtype
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((3001, 7, 5)) * 10).astype(npdt)
    b = (rng.standard_normal(5) * 3).astype(npdt)
    want = engine.run_program(prog, [torch.from_numpy(x), torch.from_numpy(b)], torch.device("cpu"))[0]
    got = engine.run_program(prog, [torch.from_numpy(x), torch.from_numpy(b)], dev)[0].cpu()
    assert "FUSED" in prog.describe([torch.from_numpy(x).to(dev), torch.from_numpy(b).to(dev)])
    if dt in (tf.int32, tf.int64):
        assert torch.equal(got, want)
    else:
        torch.testing.assert_close(got, want, rtol=1e-5 if dt == tf.float32 else 1e-12, atol=1e-6)


@pytest.mark.gpu
def test_kmeans_fused_matches_oracle_gpu():
    dev = _gpu()
    gb, c = _kmeans_graph()
    prog = engine.program(gb, ["indexes", "min_distances", "d"], ["features"])
    x = np.random.default_rng(2).uniform(size=(20011, 100))
    want = engine.run_program(prog, [torch.from_numpy(x)], torch.device("cpu"))
    got = [t.cpu() for t in engine.run_program(prog, [torch.from_numpy(x)], dev)]
    assert torch.equal(got[0], want[0])  # argmin indices
    torch.testing.assert_close(got[1], want[1], rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(got[2], want[2], rtol=1e-12, atol=1e-9)
    ref = ((x ** 2).sum(1)[:, None] + (c ** 2).sum(1)[None, :] - 2 * x @ c.T)
    np.testing.assert_array_equal(got[0].numpy(), ref.argmin(1))


@pytest.mark.gpu
@pytest.mark.parametrize("inner", [3, 16, 17, 100, 1000])
@pytest.mark.parametrize("op", ["Sum", "Mean", "Min", "Max", "Prod", "ArgMin", "ArgMax"])
def test_row_reduction_with_prologue_gpu(op, inner):
    dev = _gpu()
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float64, [None, inner], name="x")
        v = tf.abs(x) * 0.5 + 0.75 if op == "Prod" else tf.square(x) - x
        fn = {"Sum": tf.reduce_sum, "Mean": tf.reduce_mean, "Min": tf.reduce_min, "Max": tf.reduce_max,
              "Prod": tf.reduce_prod, "ArgMin": tf.argmin, "ArgMax": tf.argmax}[op]
        fn(v, 1, name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    xv = np.random.default_rng(3).standard_normal((4099, inner))
    xv[5, :] = 0.25  # ties: the first index wins
    plan = prog.describe([torch.from_numpy(xv).to(dev)])
    assert "FUSED-ROWRED" in plan, plan
    want = engine.run_program(prog, [torch.from_numpy(xv)], torch.device("cpu"))[0]
    got = engine.run_program(prog, [torch.from_numpy(xv)], dev)[0].cpu()
    if op.startswith("Arg"):
        assert torch.equal(got, want)
    else:
        torch.testing.assert_close(got, want, rtol=1e-11, atol=1e-11)


@pytest.mark.gpu
def test_uint8_image_normalisation_fuses_gpu():
    """uint8 pixels -> float normalisation in one kernel (the reference decodes
    images to uint8: src/main/python/tensorframes_snippets/read_image.py:42)."""
    dev = _gpu()
    g = tf.Graph()
    with g.as_default():
        img = tf.placeholder(tf.uint8, [None, 32, 32, 3], name="img")
        mean = tf.constant(np.array([0.485, 0.456, 0.406], np.float32))
        y = (tf.cast(img, tf.float32) / 255.0 - mean) * 2.0
        tf.identity(y, name="y")
    prog = engine.program(g.serialize(), ["y"], ["img"])
    x = np.random.default_rng(4).integers(0, 256, size=(257, 32, 32, 3), dtype=np.uint8)
    assert "FUSED" in prog.describe([torch.from_numpy(x).to(dev)])
    got = engine.run_program(prog, [torch.from_numpy(x)], dev)[0].cpu().numpy()
    want = (x.astype(np.float32) / 255.0 - np.array([0.485, 0.456, 0.406], np.float32)) * 2.0
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6)

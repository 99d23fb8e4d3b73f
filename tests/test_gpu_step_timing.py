"""Per-step device timing of the executed plan (executor set_step_timing,
utils/profiling.step_profile): every step of a GPU plan run gets a hipEvent
pair; conv / GEMM steps carry their FLOPs and the algorithm they ran
(Winograd, implicit GEMM, sibling-fused); nothing is recorded while off."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.utils.profiling import step_profile  # noqa: E402

DEV = torch.device("cuda", 0)


def test_step_profile_rows(tmp_path):
    rng = np.random.default_rng(0)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 20, 20, 16], name="x")
        y = tf.nn.relu(tf.nn.conv2d(x, tf.constant(rng.standard_normal((3, 3, 16, 32)).astype(np.float32)),
                                    [1, 1, 1, 1], "SAME"), name="c1")
        z = tf.nn.conv2d(y, tf.constant(rng.standard_normal((1, 1, 32, 8)).astype(np.float32)), [1, 2, 2, 1],
                         "VALID", name="c2")
        tf.reduce_sum(z, [1, 2, 3], name="s")
    prog = engine.program(g.serialize(), ["s"], ["x"])
    xin = torch.randn(8, 20, 20, 16, device=DEV)
    engine.run_program(prog, [xin], DEV)
    torch.cuda.synchronize()
    rows = step_profile(lambda: engine.run_program(prog, [xin], DEV), str(tmp_path / "p.json"), "t")
    by = {r["node"]: r for r in rows}
    c1 = next(r for r in rows if r["op"] == "Conv2D" and r["flops"] == 2 * 8 * 20 * 20 * 32 * 9 * 16)
    assert c1["ms"] > 0 and c1["algo"] in ("wino_f23", "implicit_gemm") and c1["calls"] == 1
    assert any(r["op"] == "Conv2D" and r["flops"] == 2 * 8 * 10 * 10 * 8 * 32 for r in rows), by
    assert abs(sum(r["share"] for r in rows) - 1.0) < 1e-6
    assert (tmp_path / "p.md").read_text().count("| Conv2D |") == 2
    # off: nothing recorded
    engine.run_program(prog, [xin], DEV)
    torch.cuda.synchronize()
    assert _C.read_step_timing() == []

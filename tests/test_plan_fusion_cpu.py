"""GPU-plan structure checked on the CPU (Program.describe(as_gpu=True) plans
for the GPU without running): pools absorb BiasAdd + Relu and write their
concat slice, nested concats are slices of the outer concat, and every
Inception-v3 mixed-block concat is written fully in place."""
import re

import numpy as np
import torch

from tensorframes_amd import engine, tf
from tensorframes_amd.models import cnn


def _plan(g, fetch, shape):
    prog = engine.program(g.serialize(), [fetch], ["x"])
    return prog.describe([torch.zeros(shape)], as_gpu=True)


def test_pool_absorbs_bias_relu_and_writes_concat_slice():
    rng = np.random.default_rng(0)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 9, 9, 16], name="x")
        a = tf.nn.relu(tf.nn.conv2d(x, tf.constant(rng.standard_normal((1, 1, 16, 8)).astype(np.float32)),
                                    [1, 1, 1, 1], "SAME"))
        p = tf.nn.avg_pool(x, [1, 3, 3, 1], [1, 1, 1, 1], "SAME")
        p = tf.nn.relu(tf.nn.bias_add(p, tf.constant(rng.standard_normal(16).astype(np.float32))))
        tf.concat([a, p], 3, name="y")
    plan = _plan(g, "y", (2, 9, 9, 16))
    pool = [l for l in plan.splitlines() if "AvgPool" in l]
    assert pool and "+bias" in pool[0] and "+relu" in pool[0] and "->concat-slice@8" in pool[0], plan
    assert "(2 inputs written in place)" in plan
    assert "FUSED" not in plan  # no separate bias/relu pass left


def test_nested_concat_is_a_slice_of_the_outer_concat():
    rng = np.random.default_rng(1)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 5, 5, 8], name="x")

        def conv(oc, kh, kw):
            w = tf.constant(rng.standard_normal((kh, kw, 8, oc)).astype(np.float32))
            return tf.nn.relu(tf.nn.conv2d(x, w, [1, 1, 1, 1], "SAME"))
        inner = tf.concat([conv(12, 1, 3), conv(12, 3, 1)], 3)
        tf.concat([conv(8, 1, 1), inner], 3, name="y")
    plan = _plan(g, "y", (2, 5, 5, 8))
    concats = [l for l in plan.splitlines() if "ConcatV2" in l]
    assert len(concats) == 2
    assert "->concat-slice@8" in concats[0] and "(2 inputs written in place)" in concats[0], plan
    assert "(2 inputs written in place)" in concats[1], plan


def test_every_inception_concat_is_written_in_place():
    g, inp, out = cnn.inception_v3(image_size=224)
    prog = engine.program(g.serialize(), [out], [inp])
    plan = prog.describe([torch.zeros((2, 224, 224, 3))], as_gpu=True)
    names = {op.name: len(op.inputs) - 1 for op in g.get_operations() if op.type == "ConcatV2"}
    seen = 0
    for line in plan.splitlines():
        m = re.search(r"OP   ConcatV2 (\S+).*\((\d+) inputs written in place\)", line)
        if m:
            seen += 1
            assert int(m.group(2)) == names[m.group(1)], line
    assert seen == len(names)

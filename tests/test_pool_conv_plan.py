"""Planner pass "pool_conv" (csrc/runtime/executor.cpp): a 3x3 VALID MaxPool
read only by a 1x1 stride-1 conv becomes part of the conv's step on GPU plans
(planned here without a GPU); any other reader, window or conv keeps the pool
step. The kernel's numerics are tests/test_gpu_pool_conv.py's."""
import numpy as np
import torch

from tensorframes_amd import engine, tf
from tensorframes_amd._native import _C


def _desc(build, gpu=True):
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 15, 15, 64], name="x")
        build(x)
    engine.clear_program_cache()
    prog = engine.program(g.serialize(), ["y"], ["x"])
    return prog.describe([torch.zeros((1, 15, 15, 64))], gpu)


def _conv(p, oc=80, k=1):
    f = np.zeros((k, k, p.get_shape().as_list()[-1], oc), np.float32)
    return tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(p, tf.constant(f), [1, 1, 1, 1], "VALID"),
                                     tf.constant(np.zeros(oc, np.float32))))


import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def fusion_on():
    _C.set_pool_conv_fusion(True)  # the default (TFA_POOL_CONV_FUSION=0 turns it off)
    yield
    _C.set_pool_conv_fusion(True)


def test_fuses_3x3_pool_into_1x1_conv():
    d = _desc(lambda x: tf.identity(_conv(tf.nn.max_pool(x, [1, 3, 3, 1], [1, 2, 2, 1], "VALID")), name="y"))
    assert "+maxpool3x3/2-in" in d and "OP   MaxPool" not in d


def test_switch_and_non_matching_shapes_keep_the_pool():
    pool = lambda x: tf.nn.max_pool(x, [1, 3, 3, 1], [1, 2, 2, 1], "VALID")  # noqa: E731
    _C.set_pool_conv_fusion(False)
    try:
        assert "-in" not in _desc(lambda x: tf.identity(_conv(pool(x)), name="y"))
    finally:
        _C.set_pool_conv_fusion(True)
    # CPU plans, a 3x3 conv, a 2x2 window, SAME padding, a second reader of the pool
    assert "-in" not in _desc(lambda x: tf.identity(_conv(pool(x)), name="y"), gpu=False)
    assert "-in" not in _desc(lambda x: tf.identity(_conv(pool(x), k=3), name="y"))
    assert "-in" not in _desc(lambda x: tf.identity(
        _conv(tf.nn.max_pool(x, [1, 2, 2, 1], [1, 2, 2, 1], "VALID")), name="y"))
    assert "-in" not in _desc(lambda x: tf.identity(
        _conv(tf.nn.max_pool(x, [1, 3, 3, 1], [1, 2, 2, 1], "SAME")), name="y"))

    def two_readers(x):
        p = pool(x)
        tf.identity(_conv(p) + tf.reduce_mean(p), name="y")
    assert "-in" not in _desc(two_readers)


def test_config_switch():
    import tensorframes_amd as tfs
    build = lambda x: tf.identity(_conv(tf.nn.max_pool(x, [1, 3, 3, 1], [1, 2, 2, 1], "VALID")), name="y")  # noqa: E731
    tfs.set_config(pool_conv_fusion=False)
    try:
        assert "-in" not in _desc(build)
        tfs.set_config(pool_conv_fusion=True)
        assert "+maxpool3x3/2-in" in _desc(build)
    finally:
        tfs.set_config(pool_conv_fusion=True)

"""Partition-task failure handling: injected faults, bounded retries, and
no retry of validation errors."""
import pytest

import tensorframes_amd as tfs
from tensorframes_amd import Row, tf
from tensorframes_amd.utils import faults
from tensorframes_amd.utils.logging import metrics


@pytest.fixture
def df():
    return tfs.create_dataframe([Row(x=float(i)) for i in range(8)], num_partitions=4)


@pytest.fixture(autouse=True)
def _retries():
    old = tfs.config.task_retries
    yield
    tfs.set_config(task_retries=old)


def _plus3(df):
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, [None], name="x")
        return tfs.map_blocks(tf.add(x, 3.0, name="z"), df)


def test_fault_fails_fast_without_retries(df):
    tfs.set_config(task_retries=0)
    with faults.inject("map_blocks", partition=2, times=1):
        with pytest.raises(faults.InjectedFault, match="partition 2"):
            _plus3(df).collect()


def test_fault_is_retried(df):
    tfs.set_config(task_retries=2)
    before = metrics.snapshot().get("task_retries", 0)
    with faults.inject("map_blocks", partition=2, times=1) as f:
        rows = _plus3(df).collect()
    assert f.times == 0
    assert [r.z for r in rows] == [i + 3.0 for i in range(8)]
    assert metrics.snapshot().get("task_retries", 0) > before


def test_persistent_fault_exhausts_retries(df):
    tfs.set_config(task_retries=2)
    with faults.inject("map_blocks", partition=1, times=10):
        with pytest.raises(faults.InjectedFault):
            _plus3(df).collect()


def test_reduce_sites_retry(df):
    tfs.set_config(task_retries=1)
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.double, [None], name="x_input")
        s = tf.reduce_sum(xi, [0], name="x")
        with faults.inject("reduce_blocks", partition=3, times=1):
            assert tfs.reduce_blocks(s, df) == 28.0
    with tf.Graph().as_default():
        a = tf.placeholder(tf.double, [], name="x_1")
        b = tf.placeholder(tf.double, [], name="x_2")
        r = tf.add(a, b, name="x")
        with faults.inject("reduce_rows", partition=0, times=1):
            assert tfs.reduce_rows(r, df) == 28.0


def test_validation_errors_are_not_retried(df):
    tfs.set_config(task_retries=3)
    assert not faults.is_retryable(tfs.TensorFramesError("bad shape"))
    assert not faults.is_retryable(ValueError("while executing node 'x': bad attr"))
    assert faults.is_retryable(ValueError("gemm: hipErrorLaunchFailure"))
    assert faults.is_retryable(RuntimeError("HIP error: an illegal memory access"))

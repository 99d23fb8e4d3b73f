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
    # sticky device faults: the context is lost, never retried in-process
    assert not faults.is_retryable(ValueError("gemm: hipErrorLaunchFailure"))
    assert not faults.is_retryable(RuntimeError("HIP error: an illegal memory access was encountered"))
    assert faults.classify(RuntimeError("Memory access fault by GPU node-2")) == "sticky"
    # deterministic HIP errors are not transient either; running out of memory is
    assert faults.classify(ValueError("HIP error invalid configuration argument in node 'y'")) == "device"
    assert not faults.is_retryable(ValueError("HIP error invalid configuration argument in node 'y'"))
    assert faults.is_retryable(RuntimeError("HIP out of memory. Tried to allocate 2.00 GiB"))
    assert faults.classify(faults.InjectedFault("x")) == "transient"


def test_sticky_fault_is_not_retried_in_process(df):
    tfs.set_config(task_retries=5)
    calls = []

    def task(blocks):
        calls.append(sorted(blocks))
        raise RuntimeError("HIP error an illegal memory access was encountered (hipErrorIllegalAddress) "
                           "in node 'y' (MatMul)")
    with pytest.raises(faults.DeviceFaultError, match="not retried in-process.*node 'y'"):
        faults.with_retries("map_blocks", task)({0: None, 1: None})
    assert len(calls) == 1  # one attempt, no per-partition re-runs


def test_oom_is_retried(df):
    tfs.set_config(task_retries=2)
    calls = []

    def task(blocks):
        calls.append(sorted(blocks))
        if len(calls) == 1:
            raise RuntimeError("HIP out of memory. Tried to allocate 64.00 GiB")
        return {p: p for p in blocks}
    assert faults.with_retries("map_blocks", task)({0: None, 1: None}) == {0: 0, 1: 1}
    assert calls == [[0, 1], [0], [1]]


def test_debug_sync_can_be_toggled_after_a_run(df):
    from tensorframes_amd._native import _C
    old = tfs.config.debug_sync
    try:
        assert [r.z for r in _plus3(df).collect()][0] == 3.0  # a program has run
        tfs.set_config(debug_sync=True)
        assert _C.get_debug_sync()
        tfs.set_config(debug_sync=False)
        assert not _C.get_debug_sync()
    finally:
        tfs.set_config(debug_sync=old)

"""Config: precision mode plumbing to the native kernel library (the GPU
numerics of each mode are in test_gpu_precision.py)."""
import pytest

import tensorframes_amd as tfs
from tensorframes_amd._native import _C


def test_precision_modes_reach_native_library():
    try:
        for name, code in (("bf16x3", 2), ("bf16", 1), ("f32", 0)):
            tfs.set_config(precision=name)
            assert _C.f32_precision() == code
    finally:
        tfs.set_config(precision="f32")


def test_bad_precision_rejected():
    with pytest.raises(ValueError):
        tfs.set_config(precision="tf32")
    tfs.set_config(precision="f32")
    with pytest.raises(Exception):
        _C.set_f32_precision(7)


def test_unknown_config_key():
    with pytest.raises(AttributeError):
        tfs.set_config(no_such_key=1)

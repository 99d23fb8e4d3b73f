"""The native JPEG decoder fails closed (csrc/runtime/jpeg_decode.cpp,
core.jpeg_native_usable): it runs only on a libjpeg whose own reported
(version, decompressor struct size) pair is a verified layout, and only after
its pixels matched the Python decoder's on a first-use self-check. A library
seen as an unknown version (jpeg_force_version, the test hook) is refused: the
decode raises, the map_rows pre-stage takes the Python decoder and counts
jpeg_native_unavailable; a self-check mismatch disables it with a warning and
jpeg_native_disabled. The GPU side (identical top-k through the pre-stage with
the library refused) is tests/test_gpu_image_prep.py."""
import io

import numpy as np
import pytest

from tensorframes_amd import core
from tensorframes_amd._native import _C
from tensorframes_amd.utils.logging import metrics

PIL = pytest.importorskip("PIL.Image")


def _jpeg():
    buf = io.BytesIO()
    PIL.fromarray(np.random.default_rng(0).integers(0, 255, (20, 30, 3), dtype=np.uint8)).save(buf, format="JPEG")
    return buf.getvalue()


@pytest.fixture
def forced():
    yield _C.jpeg_force_version
    _C.jpeg_force_version(0)
    core._JPEG_CHECKED.clear()


def test_library_reports_a_known_layout():
    info = _C.jpeg_native_info()
    if not info["ok"]:
        pytest.skip(f"no native libjpeg here: {info['why']}")
    # the version and size come from the library's own error reports
    assert info["version"] >= 60 and info["struct_size"] > 400
    assert info["soname"].startswith("libjpeg")
    assert core.jpeg_native_usable()


def test_unknown_version_is_refused(forced):
    if not _C.jpeg_native_info()["ok"]:
        pytest.skip("no native libjpeg here")
    forced(99)
    info = _C.jpeg_native_info()
    assert not info["ok"] and "unknown libjpeg layout (version 99" in info["why"], info
    assert _C.jpeg_native_available()[0] is False
    assert not core.jpeg_native_usable()
    with pytest.raises(Exception, match="unknown libjpeg layout"):
        _C.jpeg_decode(_jpeg(), 3)
    forced(0)
    assert _C.jpeg_native_info()["ok"] and core.jpeg_native_usable()
    assert np.array_equal(_C.jpeg_decode(_jpeg(), 3).numpy(), core.host_ops.decode_image(_jpeg(), 3))


def test_self_check_mismatch_disables_with_warning(forced, monkeypatch):
    if not _C.jpeg_native_info()["ok"]:
        pytest.skip("no native libjpeg here")
    core._JPEG_CHECKED.clear()
    monkeypatch.setattr(core, "_jpeg_self_check", lambda: (False, "pixels differ (simulated)"))
    metrics.reset()
    with pytest.warns(RuntimeWarning, match="native JPEG decode disabled"):
        assert not core.jpeg_native_usable()
    assert not core.jpeg_native_usable()  # cached per library: one warning
    assert metrics.snapshot()["jpeg_native_disabled"] == 1


def test_self_check_passes_on_this_library():
    if not _C.jpeg_native_info()["ok"]:
        pytest.skip("no native libjpeg here")
    assert core._jpeg_self_check() == (True, "")

"""The shipped gfx950 default tile table (tensorframes_amd/tiles/gfx950.json,
built by scripts/tile_table.py from the BASELINE workloads): well-formed keys
for the autotuner (kernels/gemm.hip tune_defaults), tiles that exist, seeded at
import. A default is replaced only by a >= 2 % win confirmed in a second timing
pass (verdict round 4, item 8)."""
import json

import pytest

from tensorframes_amd import _native
from tensorframes_amd._native import _C


def test_table_is_seeded_and_well_formed():
    entries = _native.default_entries()
    assert entries, "tensorframes_amd/tiles/gfx950.json is missing or empty"
    assert _native.TILE_DEFAULTS == len(entries)
    n = _C.gemm_tile_count()
    for e in entries:
        assert len(e["key"]) == 20 and all(isinstance(v, int) for v in e["key"])
        assert 0 <= e["tile"] < n
        bm, bn, core = _C.gemm_tile_dims(e["tile"])
        assert e["dims"] == [bm, bn] and e["core"] == ("g2" if core == 2 else "round4")
    # the headline MatMul chunk (2.5M x 512 x 512) is in it
    assert any(e["key"][:3] == [2500000, 512, 512] for e in entries)


def test_seed_rejects_bad_entries():
    with pytest.raises(Exception):
        _C.gemm_tune_seed([1, 2, 3], 0)
    with pytest.raises(Exception):
        _C.gemm_tune_seed([0] * 20, _C.gemm_tile_count())


def test_dump_merges(tmp_path):
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"entries": [{"key": [1] * 20, "tile": 3, "dims": [64, 64], "core": "round4"}]}))
    _native._dump_tune_table(str(p))
    got = json.loads(p.read_text())
    assert got["arch"] == "gfx950" and [1] * 20 in [e["key"] for e in got["entries"]]


def test_table_seeded_only_on_its_arch(monkeypatch):
    """gfx950.json is not seeded on another GPU: its tiles
    were timed on gfx950. No GPU (this container) or a gfx950 seeds it."""
    monkeypatch.setattr(_native, "_kfd_archs", lambda: {"gfx942"})
    assert _native._seed_tile_defaults() == 0
    monkeypatch.setattr(_native, "_kfd_archs", lambda: {"gfx950"})
    assert _native._seed_tile_defaults() == len(_native.default_entries())
    monkeypatch.setattr(_native, "_kfd_archs", lambda: set())
    assert _native._seed_tile_defaults() == len(_native.default_entries())

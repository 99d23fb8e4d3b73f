"""Native Row -> column packer (runtime/packer.cpp): the boxed conversion
path of create_dataframe (reference: TFDataOps.convert / DataOps.convertFast0,
src/main/scala/org/tensorframes/impl/DataOps.scala:63-81; perf case
src/test/scala/org/tensorframes/perf/ConvertPerformanceSuite.scala:19-39)."""
import time

import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import Row
from tensorframes_amd._native import _C
from tensorframes_amd.utils import dtypes as D


def test_pack_scalars_and_lists():
    rows = [(1, 2.5, [1.0, 2.0], [[1, 2], [3, 4]]), (3, 4.5, [3.0, 4.0], [[5, 6], [7, 8]])]
    a = _C.pack_column(rows, 0, 4, 0, 2, D.DT_INT64)
    assert a.dtype == torch.int64 and a.tolist() == [1, 3]
    b = _C.pack_column(rows, 1, 4, 0, 2, D.DT_FLOAT)
    assert b.dtype == torch.float32 and b.tolist() == [2.5, 4.5]
    c = _C.pack_column(rows, 2, 4, 1, 2, D.DT_DOUBLE)
    assert c.shape == (1, 2) and c.tolist() == [[3.0, 4.0]]
    d = _C.pack_column(rows, 3, 4, 0, 2, D.DT_INT32)
    assert d.shape == (2, 2, 2) and d.tolist() == [[[1, 2], [3, 4]], [[5, 6], [7, 8]]]
    # ints into a double column convert; floats into an int column do not (generic path)
    assert _C.pack_column(rows, 0, 4, 0, 2, D.DT_DOUBLE).tolist() == [1.0, 3.0]
    assert _C.pack_column(rows, 1, 4, 0, 2, D.DT_INT64) is None


def test_pack_ragged_and_errors():
    ragged = [([1.0],), ([1.0, 2.0],)]
    assert _C.pack_column(ragged, 0, 1, 0, 2, D.DT_DOUBLE) is None  # ragged: generic path
    with pytest.raises(ValueError, match="null"):
        _C.pack_column([(1.0,), (None,)], 0, 1, 0, 2, D.DT_DOUBLE)
    with pytest.raises(ValueError, match="width"):
        _C.pack_column([(1.0,), (1.0, 2.0)], 0, 1, 0, 2, D.DT_DOUBLE)
    assert _C.pack_column([("a",)], 0, 1, 0, 1, D.DT_DOUBLE) is None


def test_create_dataframe_uses_packer_and_keeps_semantics():
    df = tfs.create_dataframe([Row(x=float(i), v=[i, i + 1]) for i in range(10)], num_partitions=3)
    blocks = df.local_blocks()
    assert all(isinstance(b.columns["x"], torch.Tensor) for b in blocks.values())
    assert df.collect()[4] == (4.0, [4, 5])
    with pytest.raises(ValueError, match="null values"):
        tfs.create_dataframe([Row(x=1.0), Row(x=None)]).local_blocks()
    with pytest.raises(ValueError, match="values, schema has"):
        tfs.create_dataframe([(1.0, 2.0), (1.0,)], ["a", "b"]).local_blocks()
    rag = tfs.create_dataframe([Row(v=[1.0]), Row(v=[1.0, 2.0])], num_partitions=1)
    assert [r.v for r in rag.collect()] == [[1.0], [1.0, 2.0]]


def test_convert_rows_throughput():
    """The reference's ConvertPerformanceSuite case (10M Row(int) cells; 3M
    here to keep the suite fast; bench/configs.py refperf times 10M)."""
    n = 3_000_000
    rows = [Row(x=i) for i in range(n)]
    tfs.create_dataframe(rows[:100], num_partitions=1).local_blocks()
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        b = tfs.create_dataframe(rows, num_partitions=1).local_blocks()[0]
        best = min(best, time.perf_counter() - t0)
    assert b.columns["x"][-1].item() == n - 1
    # round 1 converted ~4M rows/s through per-value Python code
    assert n / best > 12e6, best


def test_pack_int32_out_of_range_and_list_rows_fall_back():
    # out of the int32 range: not silently truncated, the generic path reports it
    assert _C.pack_column([(1,), (1 << 40,)], 0, 1, 0, 2, D.DT_INT32) is None
    # rows that are lists, not tuples: the generic path normalises them
    assert _C.pack_column([(1.0,), [2.0]], 0, 1, 0, 2, D.DT_DOUBLE) is None
    df = tfs.create_dataframe([(1.0, 2), [3.0, 4]], ["a", "b"], num_partitions=1)
    assert df.collect() == [(1.0, 2), (3.0, 4)]


# ------------------------------------------------------------------ columns -> Rows
def test_build_rows_types_shapes_and_order():
    """Native convertBack (runtime/packer.cpp build_rows): scalars, nested
    lists for array cells, pass-through value lists, partition order."""
    x = np.arange(5, dtype=np.int32)
    f = np.linspace(0, 1, 5).astype(np.float32)
    m = np.arange(20, dtype=np.float64).reshape(5, 2, 2)
    df = tfs.from_columns({"x": x, "f": f, "m": m}, num_partitions=3)
    rows = df.collect()
    assert [type(r).__name__ for r in rows] == ["Row"] * 5 and all(isinstance(r, Row) for r in rows)
    assert [r.x for r in rows] == list(range(5)) and all(type(r.x) is int for r in rows)
    assert [r.f for r in rows] == f.tolist() and all(type(r.f) is float for r in rows)
    assert rows[3].m == [[12.0, 13.0], [14.0, 15.0]]
    assert rows[2].asDict() == {"x": 2, "f": f.tolist()[2], "m": [[8.0, 9.0], [10.0, 11.0]]}
    assert rows[0] == (0, 0.0, [[0.0, 1.0], [2.0, 3.0]])  # positional equality
    s = tfs.create_dataframe([Row(k="a", v=1.0), Row(k="b", v=2.0)], num_partitions=2).collect()
    assert s == [("a", 1.0), ("b", 2.0)] and s[1].k == "b"
    assert not hasattr(rows[0], "__dict__") or not rows[0].__dict__  # no per-row dict


def test_collect_rows_throughput():
    """The reference's ConvertBackPerformanceSuite case (10M Int cells ->
    Rows; 2M here to keep the suite fast, bench/configs.py refperf times 10M).
    Round 2 built Rows in Python at 0.36M rows/s; pinned at >= 20x that."""
    import gc
    n = 2_000_000
    df = tfs.from_columns({"x": np.arange(n, dtype=np.int32)}, num_partitions=2).cache()
    df.local_blocks()
    best = 1e9
    for _ in range(6):  # best of several: the suite may share the CPUs with other workers
        gc.collect()
        t0 = time.perf_counter()
        rows = df.collect()
        best = min(best, time.perf_counter() - t0)
        assert len(rows) == n and rows[-1].x == n - 1
        del rows
    assert n / best > 7.2e6, n / best

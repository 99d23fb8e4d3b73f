"""Arrow / Parquet interop: type mapping (primitive, nested fixed-size
lists, variable lists -> dense or ragged, strings, binary), metadata round
trip, lazy row-group partitioning, and frames from Parquet feeding graphs."""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import tf


def _table(n=10):
    rng = np.random.default_rng(0)
    mat = rng.standard_normal((n, 2, 3)).astype(np.float32)
    vec = pa.FixedSizeListArray.from_arrays(pa.array(mat.reshape(-1)), 3)
    vec = pa.FixedSizeListArray.from_arrays(vec, 2)
    return pa.table({
        "x": pa.array(np.arange(n, dtype=np.float64)),
        "k": pa.array(np.arange(n, dtype=np.int64) % 3),
        "m": vec,
        "ragged": pa.array([[float(j) for j in range(i % 4 + 1)] for i in range(n)]),
        "even": pa.array([[i, i + 1] for i in range(n)], type=pa.list_(pa.int32())),
        "s": pa.array([f"r{i}" for i in range(n)]),
        "b": pa.array([bytes([i]) * 3 for i in range(n)], type=pa.binary()),
    }), mat


def test_from_arrow_types_and_shapes():
    t, mat = _table()
    df = tfs.from_arrow(t, num_partitions=3)
    assert df.num_partitions == 3
    blocks = df.local_blocks()
    assert blocks[0].columns["m"].shape[1:] == (2, 3)
    assert blocks[0].columns["even"].dtype == torch.int32
    rows = df.collect()
    np.testing.assert_array_equal(np.asarray(rows[4].m, dtype=np.float32), mat[4])
    assert list(rows[5].ragged) == [0.0, 1.0]
    assert rows[2].s == "r2" and bytes(rows[2].b) == bytes([2]) * 3
    # metadata from fixed-size lists: block placeholders need no analyze()
    with tf.Graph().as_default():
        assert tfs.block(df, "m").get_shape().as_list() == [None, 2, 3]


def test_nulls_rejected():
    with pytest.raises(ValueError, match="null"):
        tfs.from_arrow(pa.table({"x": pa.array([1.0, None])}))


def test_arrow_roundtrip_keeps_metadata():
    t, _ = _table()
    df = tfs.analyze(tfs.from_arrow(t, num_partitions=2).select("x", "m", "even"))
    back = tfs.from_arrow(df.to_arrow(), num_partitions=2)
    assert back.schema == df.schema
    assert [r.x for r in back.collect()] == [r.x for r in df.collect()]


def test_parquet_partitions_row_groups_and_feeds_graphs(tmp_path):
    t, mat = _table(40)
    f = str(tmp_path / "data.parquet")
    pq.write_table(t, f, row_group_size=8)  # 5 row groups
    df = tfs.read_parquet(f, columns=["x", "m"])
    assert df.num_partitions == 1  # world 1: one partition unless asked
    df4 = tfs.read_parquet(f, columns=["x", "m"], num_partitions=4)
    sizes = sorted(b.nrows for b in df4.local_blocks().values())
    assert sum(sizes) == 40 and len(sizes) == 4
    with tf.Graph().as_default():
        m = tfs.block(df4, "m")
        s = tf.reduce_sum(m, [1, 2], name="s")
        out = tfs.map_blocks(s, df4)
        got = np.asarray([r.s for r in out.collect()], dtype=np.float32)
    np.testing.assert_allclose(got, mat.sum((1, 2)), rtol=1e-5)


def test_write_parquet_roundtrip(tmp_path):
    df = tfs.analyze(tfs.create_dataframe([tfs.Row(x=float(i), v=[float(i), 2.0 * i]) for i in range(9)],
                                          num_partitions=3))
    path = df.write_parquet(str(tmp_path / "out"))
    back = tfs.read_parquet(path, num_partitions=3)
    assert back.schema == df.schema
    assert [(r.x, list(r.v)) for r in back.collect()] == [(r.x, list(r.v)) for r in df.collect()]

"""DataFrame checkpoints: dense, ragged, object/binary columns and analyze
metadata survive a write/read round trip; a resumed K-Means continues from
checkpointed centers."""
import os

import numpy as np
import pytest
import torch

import tensorframes_amd as tfs
from tensorframes_amd import Row, tf


def test_roundtrip_all_column_kinds(tmp_path):
    df = tfs.create_dataframe(
        [Row(x=float(i), v=[float(i)] * (1 + i % 3), s=f"s{i}", b=bytearray(bytes([i, 255 - i])),
             m=[[i, i + 1], [i + 2, i + 3]]) for i in range(7)], num_partitions=3)
    df = tfs.analyze(df)
    path = df.write_checkpoint(str(tmp_path / "ck"))
    assert os.path.exists(os.path.join(path, "_SUCCESS"))
    back = tfs.read_checkpoint(path)
    assert back.schema == df.schema
    assert back.num_partitions == 3
    got, want = back.collect(), df.collect()
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.x == w.x and g.s == w.s and bytes(g.b) == bytes(w.b)
        np.testing.assert_array_equal(np.asarray(g.v), np.asarray(w.v))
        np.testing.assert_array_equal(np.asarray(g.m), np.asarray(w.m))
    # the analyzed metadata still drives block placeholders
    with tf.Graph().as_default():
        assert tfs.block(back, "m").get_shape().as_list() == [None, 2, 2]


def test_checkpoint_of_computed_column(tmp_path):
    df = tfs.create_dataframe([Row(x=float(i)) for i in range(10)], num_partitions=2)
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, [None], name="x")
        df2 = tfs.map_blocks(tf.multiply(x, 2.0, name="y"), df)
    back = tfs.read_checkpoint(df2.write_checkpoint(str(tmp_path / "y")))
    assert [r.y for r in back.collect()] == [2.0 * i for i in range(10)]
    with tf.Graph().as_default():
        yi = tf.placeholder(tf.double, [None], name="y_input")
        assert tfs.reduce_blocks(tf.reduce_sum(yi, [0], name="y"), back.select("y")) == 90.0


def test_incomplete_checkpoint_is_rejected(tmp_path):
    os.makedirs(tmp_path / "bad")
    with pytest.raises(FileNotFoundError):
        tfs.read_checkpoint(str(tmp_path / "bad"))


def test_kmeans_resume_from_checkpoint(tmp_path):
    from tensorframes_amd.models import kmeans
    rng = np.random.default_rng(3)
    pts = rng.uniform(0, 1, (2000, 8))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=2))
    c0 = pts[:4].copy()
    full, _ = kmeans.kmeans(df, c0, num_iters=4, tf_aggregate=True)
    # run 2 iterations, checkpoint data + centers, "restart", run 2 more
    c2, _ = kmeans.kmeans(df, c0, num_iters=2, tf_aggregate=True)
    ck = str(tmp_path / "km")
    df.write_checkpoint(ck)
    np.save(os.path.join(ck, "centers.npy"), c2)
    df_r = tfs.read_checkpoint(ck)
    c_r = np.load(os.path.join(ck, "centers.npy"))
    resumed, _ = kmeans.kmeans(df_r, c_r, num_iters=2, tf_aggregate=True)
    np.testing.assert_allclose(resumed, full, rtol=1e-12, atol=1e-12)

"""Per-key harmonic mean via map_blocks + aggregate + map_blocks
(reference: src/main/python/tensorframes_snippets/geom_mean.py:13-49)."""
from __future__ import annotations

from .. import core
from ..graph import dsl as tf


def harmonic_mean(df, col_name: str = "x", col_key: str = "key"):
    """Returns a DataFrame [key, harmonic_mean] with harmonic_mean = count / sum(1/x)."""
    with tf.Graph().as_default():
        x = core.block(df, col_name)
        invs = tf.inv(tf.to_double(x), name="invs")
        df2 = core.map_blocks([invs, tf.ones_like(invs, name="count")], df)
    gb = df2.select(col_key, "invs", "count").groupBy(col_key)
    with tf.Graph().as_default():
        x_input = core.block(df2, "invs", tf_name="invs_input")
        count_input = core.block(df2, "count", tf_name="count_input")
        x = tf.reduce_sum(x_input, [0], name="invs")
        count = tf.reduce_sum(count_input, [0], name="count")
        df3 = core.aggregate([x, count], gb)
    with tf.Graph().as_default():
        invs = core.block(df3, "invs")
        count = core.block(df3, "count")
        hm = tf.div(tf.to_double(count), invs, name="harmonic_mean")
        df4 = core.map_blocks(hm, df3).select(col_key, "harmonic_mean")
    return df4

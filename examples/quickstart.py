"""The README walk-through: map_blocks, map_rows, reduce_rows, reduce_blocks,
analyze / print_schema, aggregate (reference: README.md:56-172).

    python examples/quickstart.py            # GPU if present, else CPU
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import Row, tf  # noqa: E402


def main():
    data = [Row(x=float(x)) for x in range(10)]
    df = tfs.create_dataframe(data)

    # map_blocks: z = x + 3, one block per partition
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")
        df2 = tfs.map_blocks(z, df)
    df2.show()

    # map_rows: the same graph written against one cell
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[], name="x")
        z = tf.add(x, 3, name="z")
        print(tfs.map_rows(z, df).take(3))

    # reduce_rows: pairwise combine of X_1 / X_2
    with tf.Graph().as_default():
        x1 = tf.placeholder(tf.double, shape=[], name="x_1")
        x2 = tf.placeholder(tf.double, shape=[], name="x_2")
        x = tf.add(x1, x2, name="x")
        print("reduce_rows sum:", tfs.reduce_rows(x, df))

    # analyze: vector columns get their shape metadata, then block-level ops
    vec = tfs.analyze(tfs.create_dataframe([Row(y=[float(y), float(-y)], z=[float(y)]) for y in range(10)]))
    tfs.print_schema(vec)
    with tf.Graph().as_default():
        y_input = tfs.block(vec, "y", tf_name="y_input")
        y = tf.reduce_sum(y_input, [0], name="y")
        z_input = tfs.block(vec, "z", tf_name="z_input")
        z = tf.reduce_min(z_input, [0], name="z")
        print("reduce_blocks:", tfs.reduce_blocks([y, z], vec))

    # aggregate: per-key reduction (groupBy)
    kv = tfs.create_dataframe([Row(key=str(i % 3), x=float(i)) for i in range(12)])
    with tf.Graph().as_default():
        x_input = tfs.block(kv, "x", tf_name="x_input")
        x = tf.reduce_sum(x_input, [0], name="x")
        print(sorted(tfs.aggregate(x, kv.groupBy("key")).collect()))


if __name__ == "__main__":
    main()

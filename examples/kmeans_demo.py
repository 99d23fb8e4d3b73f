"""K-Means with TensorFrames operators (reference:
src/main/python/tensorframes_snippets/kmeans_demo.py): each iteration is a
map_blocks (distances + argmin on the GPU) followed by either an `aggregate`
over the closest-center key or an in-graph `unsorted_segment_sum` reduced
with reduce_blocks.

    python examples/kmeans_demo.py [--rows N] [--features F] [--k K] [--iters I]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    pts = rng.uniform(0, 1, (a.rows, a.features))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4)).cache()
    c0 = rng.standard_normal((a.k, a.features))
    for agg in (False, True):
        t0 = time.perf_counter()
        centers, dists = kmeans.kmeans(df, c0, num_iters=a.iters, tf_aggregate=agg)
        dt = (time.perf_counter() - t0) / a.iters
        ref_c, ref_d = c0, None
        for _ in range(a.iters):
            ref_c, ref_d = kmeans.numpy_step(pts, ref_c)
        # the in-graph variant maps an empty cluster to the origin (sums / (count + 1e-7),
        # like the reference); the aggregate variant and numpy keep its old center
        print(f"{'in-graph segment sum' if agg else 'aggregate'}: {dt * 1e3:.1f} ms/iter, "
              f"final total distance {dists[-1]:.3f} (numpy {ref_d:.3f})")


if __name__ == "__main__":
    main()

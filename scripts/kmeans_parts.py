"""Host-side breakdown of one K-Means iteration (run_one_step2, 100k x 100
f64, k = 10, device-cached): DSL graph build, serialization, native parse /
analysis / planning, and the whole iteration. VERDICT r2 item 6."""
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import core, engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.models import kmeans  # noqa: E402

gpu = torch.cuda.is_available()
dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
rng = np.random.default_rng(2)
n = 100_000 if gpu else 2_000
pts = rng.uniform(0.0, 1.0, size=(n, 100))
df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=4))
df = df.cache_on_device(dev) if gpu else df.cache()
c = rng.standard_normal((10, 100))
parts = [b.columns["features"] for _, b in sorted(df.local_blocks().items())]
T = {}
NS = {"plan_ms": 0.0, "exec_ms": 0.0}


def tick(k, t0):
    T[k] = T.get(k, 0.0) + time.perf_counter() - t0


N = 200
for it in range(N + 20):
    if it == 20:
        T.clear()
    t0 = time.perf_counter()
    g = tf.Graph()
    with g.as_default():
        points = tf.placeholder(tf.double, shape=[None, 100], name="features")
        distances = kmeans.tf_compute_distances(points, c)
        indexes = tf.argmin(distances, 1, name="indexes")
        min_distances = tf.reduce_min(distances, 1, name="min_distances")
        num_points = tf.stack([tf.shape(points)[0]], name="num_points")
        counts = tf.tile(tf.constant([1]), num_points, name="count")
        bp = tf.unsorted_segment_sum(points, indexes, 10, name="block_points")
        bc = tf.unsorted_segment_sum(counts, indexes, 10, name="block_counts")
        bd = tf.reduce_sum(min_distances, name="block_distances")
        f = [tf.expand_dims(bp, 0, name="agg_points"), tf.expand_dims(bc, 0, name="agg_counts"),
             tf.expand_dims(bd, 0, name="agg_distances")]
    tick("dsl_build_map_graph", t0)
    t0 = time.perf_counter()
    spec = core._resolve(f)
    tick("serialize", t0)
    t0 = time.perf_counter()
    gr = _C.Graph(spec.graph_bytes)
    tick("native_parse", t0)
    t0 = time.perf_counter()
    _C.analyze_fetches(gr, spec.fetch_refs, list(gr.placeholders()), {})
    tick("analyze_fetches", t0)
    t0 = time.perf_counter()
    p = _C.Program(gr, spec.fetch_refs, ["features"])
    tick("program_ctor", t0)
    t0 = time.perf_counter()
    p.row_separable({"features": (2, [-1, 100])})
    tick("row_separable", t0)
    t0 = time.perf_counter()
    for x in parts:
        p.run([x])
    tick("run_4_partitions", t0)
    st = p.stats()
    for k in NS:
        NS[k] += st[k]
if gpu:
    torch.cuda.synchronize()
res = {k: v / N * 1e6 for k, v in T.items()}
res.update({"native_" + k: v / N * 1e3 for k, v in NS.items()})
for _ in range(5):
    c, _ = kmeans.run_one_step2(df, c)
if gpu:
    torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    c, _ = kmeans.run_one_step2(df, c)
if gpu:
    torch.cuda.synchronize()
res["iteration_us"] = (time.perf_counter() - t0) / N * 1e6
print(json.dumps({"us": res, "gpu": gpu}), flush=True)
out = sys.argv[1] if len(sys.argv) > 1 else None
if out:
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        c, _ = kmeans.run_one_step2(df, c)
    pr.disable()
    with open(out, "w") as fh:
        st = pstats.Stats(pr, stream=fh)
        st.sort_stats("tottime").print_stats(40)
        st.sort_stats("cumulative").print_stats(60)

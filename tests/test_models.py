"""Workloads of the reference's snippets: K-Means (both variants) and the
per-key harmonic mean, checked against numpy oracles."""
import numpy as np

import tensorframes_amd as tfs
from tensorframes_amd import Row
from tensorframes_amd.models import harmonic_mean, kmeans


def _points(n=600, f=5, seed=2):
    rng = np.random.default_rng(seed)
    return rng.uniform(0.0, 1.0, size=(n, f))


def test_kmeans_one_step_aggregate_matches_numpy():
    pts = _points()
    c0 = np.random.default_rng(3).standard_normal((4, 5))
    df = tfs.analyze(tfs.create_dataframe([[list(p)] for p in pts], ["features"], num_partitions=3))
    got_c, got_d = kmeans.run_one_step(df, c0)
    want_c, want_d = kmeans.numpy_step(pts, c0)
    np.testing.assert_allclose(got_c, want_c, rtol=1e-10, atol=1e-10)
    assert abs(got_d - want_d) < 1e-8 * max(1, want_d)


def test_kmeans_one_step_in_graph_aggregation_matches_numpy():
    pts = _points()
    c0 = np.random.default_rng(3).standard_normal((4, 5))
    df = tfs.analyze(tfs.create_dataframe([[list(p)] for p in pts], ["features"], num_partitions=3))
    got_c, got_d = kmeans.run_one_step2(df, c0)
    want_c, want_d = kmeans.numpy_step(pts, c0)
    # empty clusters become 0 / (0 + 1e-7) = 0 in this variant (as in the reference demo)
    d = (pts ** 2).sum(1)[:, None] + (c0 ** 2).sum(1)[None, :] - 2 * pts @ c0.T
    nonempty = np.bincount(d.argmin(1), minlength=4) > 0
    np.testing.assert_allclose(got_c[nonempty], want_c[nonempty], rtol=1e-6, atol=1e-6)
    assert (got_c[~nonempty] == 0).all()
    assert abs(got_d - want_d) < 1e-8 * max(1, want_d)


def test_kmeans_runs_and_decreases():
    pts = _points(300, 3)
    c0 = pts[:3].copy()
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=2))
    c, ds = kmeans.kmeans(df, c0, num_iters=4, tf_aggregate=True)
    assert c.shape == (3, 3)
    assert all(b <= a + 1e-9 for a, b in zip(ds, ds[1:]))


def test_harmonic_mean():
    data = [Row(x=[float(x), float(2 * x)], key=str(x % 2)) for x in range(1, 6)]
    df = tfs.analyze(tfs.create_dataframe(data))
    rows = harmonic_mean.harmonic_mean(df).collect()
    by = {r.key: r.harmonic_mean for r in rows}
    for key in ("0", "1"):
        xs = np.array([[x, 2 * x] for x in range(1, 6) if str(x % 2) == key], dtype=np.float64)
        want = len(xs) / (1.0 / xs).sum(0)
        np.testing.assert_allclose(by[key], want)

"""Is F(4x4,3x3) accurate enough in f32? (round-5 verdict: "evaluate
F(4x4,3x3)"). Emulates, in float32 numpy, the direct convolution (the exact
implicit-GEMM path), Winograd F(2x2,3x3) (what conv_wino.hip runs: filter
transform in fp64 rounded once, input / output transforms in f32) and
F(4x4,3x3) (points 0, +-1, +-2, inf; Lavin & Gray 2016), on Inception-v3 /
VGG-16 layer shapes with ReLU-like (non-negative) and signed inputs, and
reports the accuracy gate of tests/test_gpu_wino.py: max |y - y64| / sum|a*b|
and the ratio to the direct path's error. The gate for a default-on path is
<= 1e-5 and <= 4x the direct error.

    python scripts/wino_precision_eval.py [--json out.json]
"""
import argparse
import json

import numpy as np

F23 = dict(
    BT=np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64),
    G=np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64),
    AT=np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64), m=2)
F43 = dict(
    BT=np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
                 [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float64),
    G=np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
                [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], np.float64),
    AT=np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], np.float64),
    m=4)


def direct(x, f, dt):
    n, h, w, c = x.shape
    oh, ow = h - 2, w - 2
    cols = np.stack([x[:, a:a + oh, b:b + ow, :] for a in range(3) for b in range(3)], 3)
    return np.einsum("nhwkc,kco->nhwo", cols.astype(dt), f.reshape(9, c, -1).astype(dt), optimize=True)


def winograd(x, f, T, dt):
    """VALID conv of x [n, h, w, c] (h - 2, w - 2 divisible by m) in dtype dt,
    the filter transform in fp64 rounded once to dt"""
    BT, G, AT, m = T["BT"], T["G"], T["AT"], T["m"]
    a = BT.shape[0]
    n, h, w, c = x.shape
    oc = f.shape[3]
    oh, ow = h - 2, w - 2
    u = np.einsum("ia,abco,jb->ijco", G, f.astype(np.float64), G).astype(dt)        # a x a x c x oc
    th, tw = oh // m, ow // m
    idx_h = (np.arange(th) * m)[:, None] + np.arange(a)[None]
    idx_w = (np.arange(tw) * m)[:, None] + np.arange(a)[None]
    d = x[:, idx_h][:, :, :, idx_w].astype(dt)                                      # n, th, a, tw, a, c
    d = d.transpose(0, 1, 3, 2, 4, 5)                                               # n, th, tw, a, a, c
    v = np.einsum("ia,ntwabc,jb->ntwijc", BT.astype(dt), d, BT.astype(dt), optimize=True).astype(dt)
    mm = np.einsum("ntwijc,ijco->ntwijo", v, u, optimize=True).astype(dt)
    y = np.einsum("pi,ntwijo,qj->ntpwqo", AT.astype(dt), mm, AT.astype(dt), optimize=True).astype(dt)
    return y.reshape(n, th * m, tw * m, oc)


def gate(y, ref, scale):
    return float(np.max(np.abs(y.astype(np.float64) - ref) / scale))


LAYERS = [  # name, n, h, w, c, oc (VALID; h - 2, w - 2 divisible by 4)
    ("Conv2d_2b-like C32 OC64", 2, 26, 26, 32, 64),
    ("Conv2d_4a-like C80 OC192", 2, 26, 26, 80, 192),
    ("Mixed_5 b2 C96 OC96", 2, 18, 18, 96, 96),
    ("Mixed_7 b2 C448 OC384", 2, 10, 10, 448, 384),
    ("VGG conv4_x C512 OC512", 1, 14, 14, 512, 512),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    # exactness of the transforms in fp64
    x = rng.uniform(-1, 1, (1, 10, 10, 4))
    f = rng.uniform(-1, 1, (3, 3, 4, 5))
    for T in (F23, F43):
        assert np.allclose(winograd(x, f, T, np.float64), direct(x, f, np.float64), atol=1e-10)
    rows = []
    for name, n, h, w, c, oc in LAYERS:
        for dist in ("relu", "signed"):
            x = rng.uniform(-1, 1, (n, h, w, c))
            if dist == "relu":
                x = np.maximum(x, 0) * rng.uniform(0.5, 2.0)
            f = rng.normal(0, np.sqrt(2.0 / (9 * c)), (3, 3, c, oc))
            ref = direct(x, f, np.float64)
            scale = direct(np.abs(x), np.abs(f), np.float64)
            e_d = gate(direct(x.astype(np.float32), f.astype(np.float32), np.float32), ref, scale)
            e_23 = gate(winograd(x.astype(np.float32), f, F23, np.float32), ref, scale)
            e_43 = gate(winograd(x.astype(np.float32), f, F43, np.float32), ref, scale)
            r = {"layer": name, "input": dist, "direct": e_d, "f23": e_23, "f43": e_43,
                 "f23_vs_direct": e_23 / e_d, "f43_vs_direct": e_43 / e_d,
                 "f43_passes_gate": e_43 <= 1e-5 and e_43 <= 4 * e_d}
            rows.append(r)
            print(f"{name:26s} {dist:6s} direct {e_d:.2e}  F(2x2,3x3) {e_23:.2e} ({e_23 / e_d:4.1f}x)  "
                  f"F(4x4,3x3) {e_43:.2e} ({e_43 / e_d:5.1f}x)  gate {'pass' if r['f43_passes_gate'] else 'FAIL'}",
                  flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()

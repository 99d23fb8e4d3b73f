"""Per-layer f32 conv throughput of Inception-v3 (the BASELINE config-5 model)
or VGG-16 (the reference's read_image network) on device-resident tensors:
every Conv2D+BiasAdd+Relu of the network, timed on its own through the engine
(autotuned tile), with its share of the total. Shows which layers hold the
network below the f32 MFMA peak. (The plan that really runs, with its fusions,
is timed per step by `--step-profile` of bench/configs.py and read_image.py.)

    python scripts/conv_layers.py [--model inception_v3|vgg16] [--batch 2048] [--image 224] [--json out.json] [--vendor]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd.models import cnn  # noqa: E402

F32_PEAK_TF = 157.3


def model_convs(image, model="inception_v3"):
    """(H, W, C, KH, KW, OC, stride, padding) of every conv, in network order."""
    seen = []
    orig = cnn._Builder.conv

    def rec(self, x, out_c, kh, kw, stride=1, padding="SAME", name=None, relu=True, scale_out=True):
        _, h, w, c = x.get_shape().as_list()
        oc = self.ch(out_c) if scale_out else out_c
        seen.append((h, w, c, kh, kw, oc, stride, padding, name))
        return orig(self, x, out_c, kh, kw, stride, padding, name, relu, scale_out)

    cnn._Builder.conv = rec
    try:
        getattr(cnn, model)(image_size=image)
    finally:
        cnn._Builder.conv = orig
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "vgg16"])
    ap.add_argument("--batch", type=int, default=None, help="default: 2048 (Inception), 256 (VGG-16)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--vendor", action="store_true", help="also time MIOpen (F.conv2d, channels_last, exact f32)")
    ap.add_argument("--only", type=int, default=-1, help="run only unique layer #i (counter runs)")
    a = ap.parse_args()
    from tensorframes_amd._native import _C
    torch.backends.cudnn.allow_tf32 = False
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    if a.batch is None:
        a.batch = 2048 if a.model == "inception_v3" else 256
    layers = model_convs(a.image, a.model)
    uniq = {}
    for l in layers:
        uniq.setdefault(l[:8], []).append(l[8])
    res, tot_ms, tot_fl = [], 0.0, 0.0
    for li, ((h, w, c, kh, kw, oc, s, pad), names) in enumerate(uniq.items()):
        if a.only >= 0 and li != a.only:
            continue
        before = {tuple(k): t for k, t in _C.gemm_tune_table()}
        g = tf.Graph()
        with g.as_default():
            x = tf.placeholder(tf.float32, [None, h, w, c], name="x")
            f = tf.constant((rng.standard_normal((kh, kw, c, oc)) * 0.05).astype(np.float32))
            y = tf.nn.conv2d(x, f, [1, s, s, 1], pad)
            tf.nn.relu(tf.nn.bias_add(y, tf.constant(np.zeros(oc, np.float32))), name="y")
        prog = engine.program(g.serialize(), ["y"], ["x"])
        xin = torch.randn((a.batch, h, w, c), device=dev)
        t0 = time.perf_counter()  # >= 0.2 s warm: clocks ramped, tile tuned
        while time.perf_counter() - t0 < 0.2:
            engine.run_program(prog, [xin], dev)
            torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            engine.run_program(prog, [xin], dev)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.iters
        oh = (h - kh) // s + 1 if pad == "VALID" else (h + s - 1) // s
        ow = (w - kw) // s + 1 if pad == "VALID" else (w + s - 1) // s
        fl = 2.0 * a.batch * oh * ow * oc * kh * kw * c
        n = len(names)
        tot_ms += ms * n
        tot_fl += fl * n
        new = [(k, t) for k, t in _C.gemm_tune_table() if tuple(k) not in before]
        tile = new[0][1] if len(new) == 1 else (None if not new else [t for _, t in new])
        dims = _C.gemm_tile_dims(tile) if isinstance(tile, int) else None
        r = {"index": li, "layer": names[0], "count": n, "H": h, "W": w, "C": c, "KH": kh, "KW": kw, "OC": oc,
             "stride": s, "pad": pad, "M": a.batch * oh * ow, "K": kh * kw * c, "ms": ms, "tflops": fl / ms / 1e9,
             "tile": tile, "tile_dims": None if dims is None else f"{dims[0]}x{dims[1]}",
             "core": None if dims is None else ("g2" if dims[2] == 2 else "round4")}
        # the algorithm that ran: the plan carries a Winograd filter for 3x3 /
        # 1x7 / 7x1 stride-1 convs (conv_wino.hip conv_wino_eligible)
        wino = "+winograd" in prog.describe([xin[:1].cpu()], True) and _C.conv_wino_enabled()
        r["algo"] = ("wino_f23" if kh == 3 else "wino_f45" if kh == 5 else "wino_f27") if wino else (
            "direct" if dims is None else f"gemm {r['core']} {r['tile_dims']}")
        if a.vendor:
            import torch.nn.functional as F
            xn = xin.permute(0, 3, 1, 2)
            wt = torch.randn((oc, c, kh, kw), device=dev).contiguous(memory_format=torch.channels_last)
            bt = torch.zeros((oc,), device=dev)
            padding = "same" if pad == "SAME" and s == 1 else 0
            if pad == "SAME" and s != 1:
                ph, pw = max((oh - 1) * s + kh - h, 0), max((ow - 1) * s + kw - w, 0)
                xn = F.pad(xn, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)).contiguous(
                    memory_format=torch.channels_last)
            fn = lambda: torch.relu(F.conv2d(xn, wt, bt, stride=s, padding=padding))  # noqa: E731
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.iters):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            vms = ev[0].elapsed_time(ev[1]) / a.iters
            r.update(vendor_ms=vms, vendor_tflops=fl / vms / 1e9)
            del xn, wt, bt
        print(json.dumps(r), flush=True)
        res.append(r)
        del xin
    for r in res:
        r["share"] = r["ms"] * r["count"] / tot_ms
    summ = {"model": a.model, "batch": a.batch, "image": a.image, "conv_ms_total": tot_ms, "conv_tflops": tot_fl / tot_ms / 1e9,
            "fraction_of_f32_peak": tot_fl / tot_ms / 1e9 / F32_PEAK_TF,
            "images_per_s_conv_only": a.batch / tot_ms * 1e3}
    print(json.dumps(summ), flush=True)
    for r in sorted(res, key=lambda r: -r["share"]):
        print(f"{r['share'] * 100:5.1f}%  {r['tflops']:6.1f} TF  {r.get('algo', ''):>18s} {r['layer']:>14s} x{r['count']}  "
              f"{r['H']}x{r['W']}x{r['C']} k{r['KH']}x{r['KW']} s{r['stride']} -> {r['OC']}  M={r['M']} K={r['K']}",
              flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"summary": summ, "layers": res}, f, indent=1)


if __name__ == "__main__":
    main()

"""Image scoring from a binary column of JPEG bytes (reference:
src/main/python/tensorframes_snippets/read_image.py): DecodeJpeg runs as a
host stage, everything after it (resize, crop, VGG-16, softmax, top-k) runs
in the native executor on the GPU, one image per row through `map_rows`.

No network here: the JPEGs are synthetic and VGG-16 has random weights.

    python examples/read_image.py [--images N] [--width W]
"""
import argparse
import io
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import Row  # noqa: E402
from tensorframes_amd.models import cnn  # noqa: E402


def synthetic_jpegs(n, rng):
    out = []
    for i in range(n):
        h, w = rng.integers(180, 400, 2)
        arr = rng.integers(0, 255, (h, w, 3), dtype=np.uint8)
        buf = io.BytesIO()
        Image.fromarray(arr).save(buf, format="JPEG", quality=90)
        out.append((f"file:/synthetic/img{i}.jpg", bytearray(buf.getvalue())))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--width", type=float, default=1.0, help="VGG channel multiplier (1.0 = VGG-16)")
    ap.add_argument("--prep", choices=["reference", "slim"], default="reference",
                    help="reference: square resize + crop (read_image.py); slim: aspect-preserving resize")
    ap.add_argument("--step-profile", default="", help="then one more pass with per-step device timing -> JSON/.md")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    imgs = synthetic_jpegs(a.images, rng)
    df = tfs.create_dataframe([Row(image_uri=u, image_data=b) for u, b in imgs])
    # the graph is built around one image, like the reference; map_rows feeds
    # the column into 'DecodeJpeg/contents' row by row
    g = cnn.jpeg_scoring_graph("vgg16", contents=bytes(imgs[0][1]), width=a.width, preprocessing=a.prep)
    with g.as_default():
        pred = tfs.map_rows(["index", "value"], df, feed_dict={"DecodeJpeg/contents": "image_data"})
        from tensorframes_amd._native import _C
        for attempt in ("first pass (plans, kernel tile tuning)", "steady state"):
            tfs.metrics.reset()
            if attempt == "steady state":
                _C.roctx_push("tfa.timed_steps")  # rocprofv3 --marker-trace: the timed window
            t0 = time.perf_counter()
            rows = pred.select("image_uri", "index", "value").collect()
            dt = time.perf_counter() - t0
            if attempt == "steady state":
                _C.roctx_pop()
            print(f"{attempt}: {len(rows)} images in {dt:.2f}s ({len(rows) / dt:.1f} images/s)")
        if a.step_profile:
            from tensorframes_amd.utils.profiling import step_profile
            step_profile(lambda: pred.select("image_uri", "index", "value").collect(), a.step_profile,
                         f"VGG-16 JPEG scoring ({a.prep} preprocessing), {a.images} images: per-step device time")
    for r in rows[:4]:
        print(r.image_uri, list(r["index"]), [round(v, 4) for v in r["value"]])
    m = tfs.metrics.snapshot()
    print({k: round(v, 1) for k, v in m.items() if k.startswith("map_rows")})
    from tensorframes_amd.utils.sysinfo import box_id
    print("box:", box_id())


if __name__ == "__main__":
    main()

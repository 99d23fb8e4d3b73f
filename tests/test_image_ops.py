"""Image preprocessing ops: ResizeBilinear / ResizeNearestNeighbor (all three
coordinate modes) against numpy references, and the DecodeJpeg/DecodePng host
stage of map_rows (binary column -> decoded uint8 image -> GPU/CPU program),
the flow of the reference's VGG scoring example
(reference: src/main/python/tensorframes_snippets/read_image.py:42,147-167)."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

import tensorframes_amd as tfs
from tensorframes_amd import engine, tf
from tensorframes_amd.core import TensorFramesError

rng = np.random.default_rng(7)


def _src(out, inp, mode):
    if mode == "align":
        s = (inp - 1) / (out - 1) if out > 1 else inp / out
        return np.arange(out) * s
    s = inp / out
    return (np.arange(out) + 0.5) * s - 0.5 if mode == "half" else np.arange(out) * s


def bilinear_ref(x, oh, ow, mode):
    n, h, w, c = x.shape
    ys, xs = _src(oh, h, mode), _src(ow, w, mode)
    y0 = np.clip(np.floor(ys), 0, h - 1).astype(int)
    y1 = np.minimum(np.ceil(ys), h - 1).astype(int)
    x0 = np.clip(np.floor(xs), 0, w - 1).astype(int)
    x1 = np.minimum(np.ceil(xs), w - 1).astype(int)
    ly = (ys - np.floor(ys))[None, :, None, None]
    lx = (xs - np.floor(xs))[None, None, :, None]
    f = x.astype(np.float64)
    top = f[:, y0][:, :, x0] + (f[:, y0][:, :, x1] - f[:, y0][:, :, x0]) * lx
    bot = f[:, y1][:, :, x0] + (f[:, y1][:, :, x1] - f[:, y1][:, :, x0]) * lx
    return top + (bot - top) * ly


def nearest_ref(x, oh, ow, mode):
    n, h, w, c = x.shape

    def idx(out, inp):
        s = (inp - 1) / (out - 1) if (mode == "align" and out > 1) else inp / out
        d = np.arange(out)
        v = np.round(d * s) if mode == "align" else (np.floor((d + 0.5) * s) if mode == "half" else np.floor(d * s))
        return np.clip(v, 0, inp - 1).astype(int)
    return x[:, idx(oh, h)][:, :, idx(ow, w)]


def run(g, fetches, feeds, device=None):
    names = list(feeds)
    prog = engine.program(g.serialize(), fetches, names)
    ins = [torch.as_tensor(np.asarray(feeds[n])) for n in names]
    return [o.cpu().numpy() for o in engine.run_program(prog, ins, device or torch.device("cpu"))]


@pytest.mark.parametrize("mode", ["legacy", "align", "half"])
@pytest.mark.parametrize("dtype", [np.uint8, np.float32])
@pytest.mark.parametrize("size", [(7, 9), (31, 17), (1, 1)])
def test_resize_modes(mode, dtype, size):
    x = (rng.random((2, 13, 11, 3)) * 255).astype(dtype)
    g = tf.Graph()
    with g.as_default():
        xi = tf.placeholder(tf.as_dtype(dtype), [None, 13, 11, 3], name="x")
        kw = dict(align_corners=mode == "align", half_pixel_centers=mode == "half")
        tf.image.resize_bilinear(xi, list(size), name="bl", **kw)
        tf.image.resize_nearest_neighbor(xi, list(size), name="nn", **kw)
    bl, nn = run(g, ["bl", "nn"], {"x": x})
    assert bl.dtype == np.float32 and nn.dtype == dtype
    np.testing.assert_allclose(bl, bilinear_ref(x, *size, mode), rtol=1e-5, atol=1e-3)
    np.testing.assert_array_equal(nn, nearest_ref(x, *size, mode))


def test_resize_shape_inference_and_resize_images_3d():
    with tf.Graph().as_default():
        x = tf.placeholder(tf.uint8, [None, None, 3], name="x")
        y = tf.image.resize_images(tf.image.convert_image_dtype(x, tf.float32), [24, 20])
        assert y.get_shape().as_list() == [24, 20, 3]
        c = tf.image.central_crop_to(y, 16, 16)
        assert c.get_shape().as_list() == [16, 16, 3]


def _encode(a, fmt):
    buf = io.BytesIO()
    Image.fromarray(a.squeeze(-1) if a.shape[-1] == 1 else a).save(buf, format=fmt)
    return buf.getvalue()


def _decoded(b, mode=None):
    im = Image.open(io.BytesIO(b))
    return np.asarray(im.convert(mode) if mode else im)


def _image_frame(fmt="PNG"):
    shapes = [(40, 52), (33, 21), (64, 64), (17, 90)]
    raw = [_encode(rng.integers(0, 255, (h, w, 3), dtype=np.uint8), fmt) for h, w in shapes]
    df = tfs.create_dataframe([tfs.Row(uri=f"img{i}", image_data=bytearray(r)) for i, r in enumerate(raw)],
                              num_partitions=2)
    return df, raw


@pytest.mark.parametrize("fmt", ["PNG", "JPEG"])
def test_map_rows_decode_host_stage(fmt):
    df, raw = _image_frame(fmt)
    with tf.Graph().as_default():
        contents = tf.placeholder(tf.string, [], name="contents")
        im = (tf.image.decode_png if fmt == "PNG" else tf.image.decode_jpeg)(contents, channels=3)
        x = tf.image.convert_image_dtype(im, tf.float32)
        r = tf.image.resize_images(x, [16, 16])
        tf.reduce_mean(r, [0, 1], name="m")
        tf.identity(tf.shape(im), name="hw")
        out = tfs.map_rows(["m", "hw"], df, feed_dict={"contents": "image_data"})
    rows = out.collect()
    assert [r.uri for r in rows] == [f"img{i}" for i in range(4)]
    for row, b in zip(rows, raw):
        a = _decoded(b, "RGB")
        assert list(row.hw) == list(a.shape)
        ref = bilinear_ref(a[None].astype(np.float64) / 255.0, 16, 16, "legacy")[0].mean((0, 1))
        np.testing.assert_allclose(np.asarray(row.m), ref, rtol=1e-5, atol=1e-6)


def test_map_rows_decode_feeds_contents_const():
    """The reference example builds the graph around a constant JPEG and feeds
    'DecodeJpeg/contents' from the column (read_image.py:39-42,165)."""
    df, raw = _image_frame("JPEG")
    with tf.Graph().as_default():
        im = tf.image.decode_jpeg(raw[0], channels=3)  # Const 'DecodeJpeg/contents'
        tf.identity(tf.reduce_sum(tf.cast(im, tf.int64)), name="s")
        out = tfs.map_rows("s", df, feed_dict={"DecodeJpeg/contents": "image_data"})
    got = [r.s for r in out.collect()]
    assert got == [int(_decoded(b, "RGB").astype(np.int64).sum()) for b in raw]
    # without the feed the constant is decoded once and used for every row
    with tf.Graph().as_default():
        im = tf.image.decode_jpeg(raw[1], channels=1)
        tf.identity(tf.reduce_sum(tf.cast(im, tf.int64)), name="s")
        out = tfs.map_rows("s", df)
    assert {r.s for r in out.collect()} == {int(_decoded(raw[1], "L").astype(np.int64).sum())}


def test_decode_requires_binary_column():
    df = tfs.create_dataframe([tfs.Row(x=1.0, image_data=bytearray(b"\x00"))])
    with tf.Graph().as_default():
        contents = tf.placeholder(tf.string, [], name="contents")
        tf.identity(tf.image.decode_png(contents, channels=3), name="img")
        with pytest.raises(TensorFramesError, match="binary column"):
            tfs.map_rows("img", df, feed_dict={"contents": "x"})


def test_decode_op_outside_host_stage_fails_loudly():
    g = tf.Graph()
    with g.as_default():
        tf.identity(tf.image.decode_png(_encode(np.zeros((4, 4, 3), np.uint8), "PNG")), name="img")
    with pytest.raises(ValueError, match="host op"):
        prog = engine.program(g.serialize(), ["img"], [])
        engine.run_program(prog, [], torch.device("cpu"))


def test_jpeg_scoring_graph_batch_cut_matches_per_row_loop():
    """The reference's read_image pipeline (DecodeJpeg host stage -> resize ->
    crop -> mean subtraction -> batch of one -> VGG -> softmax -> top_k of the
    squeezed probabilities): the batch-of-one cut gives the per-row results."""
    from tensorframes_amd.models import cnn
    from tensorframes_amd.utils.logging import metrics
    df, raw = _image_frame("JPEG")
    g = cnn.jpeg_scoring_graph("vgg16", image_size=32, contents=raw[0], width=0.0625, fc_width=32, k=3)
    outs = {}
    old = tfs.config.map_rows_vectorize
    try:
        for vec in (True, False):
            tfs.set_config(map_rows_vectorize=vec)
            metrics.reset()
            with g.as_default():
                res = tfs.map_rows(["index", "value"], df, feed_dict={"DecodeJpeg/contents": "image_data"})
                rows = res.collect()
            outs[vec] = ([list(r["index"]) for r in rows], np.array([list(r["value"]) for r in rows]))
            cut_rows = metrics.snapshot().get("map_rows_batch_cut_rows", 0)
            assert (cut_rows == len(raw)) if vec else cut_rows == 0
    finally:
        tfs.set_config(map_rows_vectorize=old)
    assert outs[True][0] == outs[False][0]
    # float32 sums in another order (batched GEMM vs per-row): probabilities to ~1e-6
    np.testing.assert_allclose(outs[True][1], outs[False][1], rtol=1e-4, atol=1e-6)

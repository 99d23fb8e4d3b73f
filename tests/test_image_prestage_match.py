"""The batched image pre-stage is recognised from the graph alone (CPU):
core._match_image_prep on the reference's JPEG scoring chain
(src/main/python/tensorframes_snippets/read_image.py:35-75: decode -> cast ->
resize -> central crop -> mean subtraction -> expand_dims) and on variants it
must take (channel count from the decoder) or refuse (ops it does not model)."""
import numpy as np
import pytest

from tensorframes_amd import core, tf
from tensorframes_amd.ops import image_prep
from tensorframes_amd.models import cnn


def _cut(g, fetches):
    spec_refs = [f"{n}:0" for n in fetches]
    bc = core._BatchCut(g.serialize(), spec_refs, ["DecodeJpeg"])
    return bc


def test_reference_chain_is_recognised():
    g = cnn.jpeg_scoring_graph("vgg16", contents=b"\xff\xd8", width=0.125)
    bc = _cut(g, ["index", "value"])
    assert bc.cut is not None
    p = bc.image_prep
    assert p is not None
    assert (p.OH, p.OW) == (256, 256) or p.OH >= p.h
    assert p.h == 224 and p.w == 224 and p.channels() == 3
    assert len(p.ops) >= 1 and p.ops[0][0] == 1  # the mean subtraction


def _chain(channels, tail, slice_c=-1):
    g = tf.Graph()
    with g.as_default():
        data = tf.placeholder(tf.string, [], name="data")
        im = tf.image.decode_jpeg(data, channels=channels, name="DecodeJpeg")
        x = tf.cast(im, tf.float32)
        x = tf.image.resize_bilinear(tf.expand_dims(x, 0), [40, 40])
        x = tf.slice(tf.squeeze(x, [0]), [4, 4, 0], [32, 32, slice_c])
        x = tail(x)
        x = tf.expand_dims(x, 0)
        c = channels or 3
        y = tf.nn.conv2d(x, tf.constant(np.ones((3, 3, c, 4), np.float32)), [1, 1, 1, 1], "SAME")
        tf.reduce_sum(tf.nn.relu(y), [1, 2], name="s")
    return g


def test_grayscale_chain_and_decoder_channels():
    g = _chain(1, lambda x: tf.multiply(x, 0.5), slice_c=1)
    p = _cut(g, ["s"]).image_prep
    assert p is not None and p.C == 1 and p.ops == [(2, [0.5])]
    # a chain that leaves the channel count open takes the decoder's
    from tensorframes_amd.ops.host_ops import HostFeed
    open_c = core._ImagePrep(None, 40, 40, 0, 4, 4, 32, 32, [])
    assert open_c.channels(HostFeed("DecodeJpeg", "DecodeJpeg", 3, 4, "c")) == 3
    assert open_c.channels(HostFeed("DecodeJpeg", "DecodeJpeg", 0, 4, "c")) is None


def test_per_channel_constants_fix_the_channel_count():
    g = _chain(3, lambda x: tf.subtract(x, tf.constant(np.array([1, 2, 3], np.float32))))
    p = _cut(g, ["s"]).image_prep
    assert p is not None and p.C == 3


def test_unmodelled_ops_are_refused():
    g = _chain(3, lambda x: tf.nn.relu(x))
    assert _cut(g, ["s"]).image_prep is None


def slim_eval_graph(side=256, crop=224, means=(123.68, 116.78, 103.94), with_cnn=True):
    """slim-style eval preprocessing (vgg_preprocessing.preprocess_for_eval):
    aspect-preserving resize of the uint8 image to smallest side `side`,
    central crop computed from the resized shape, per-channel mean
    subtraction through split / concat, then a batch of one."""
    g = tf.Graph()
    with g.as_default():
        data = tf.placeholder(tf.string, [], name="data")
        im = tf.image.decode_jpeg(data, channels=3, name="DecodeJpeg")
        shp = tf.shape(im)
        hf, wf = tf.cast(shp[0], tf.float32), tf.cast(shp[1], tf.float32)
        scale = tf.where(tf.greater(hf, wf), float(side) / wf, float(side) / hf)
        nh = tf.cast(tf.round(hf * scale), tf.int32, name="new_h")
        nw = tf.cast(tf.round(wf * scale), tf.int32, name="new_w")
        x = tf.squeeze(tf.image.resize_bilinear(tf.expand_dims(im, 0), [nh, nw]))
        rs = tf.shape(x)
        oy = tf.identity((rs[0] - crop) // 2, name="off_h")
        ox = tf.identity((rs[1] - crop) // 2, name="off_w")
        x = tf.slice(x, [oy, ox, 0], [crop, crop, 3])
        x = tf.cast(x, tf.float32)
        r, gch, b = tf.split(x, 3, axis=2)
        x = tf.concat([r - means[0], gch - means[1], b - means[2]], 2)
        x = tf.expand_dims(x, 0, name="prepped")
        if with_cnn:
            y = tf.nn.conv2d(x, tf.constant(np.ones((3, 3, 3, 4), np.float32) * 1e-3), [1, 1, 1, 1], "SAME")
            tf.reduce_sum(tf.nn.relu(y), [1, 2], name="s")
    return g


def test_slim_style_chain_is_recognised_with_per_row_sizes():
    g = slim_eval_graph()
    bc = _cut(g, ["s"])
    assert bc.cut == "prepped"
    p = bc.image_prep
    assert p is not None and p.dyn is not None
    assert (p.h, p.w, p.C, p.mode) == (224, 224, 3, 0)
    assert p.ops == [(1, [np.float32(123.68), np.float32(116.78), np.float32(103.94)])]


def test_per_row_sizes_match_the_cpu_executor():
    """The host evaluation of the shape-only part gives, for every image
    size, the resize size and crop offset the graph itself computes on the
    CPU executor."""
    import torch

    from tensorframes_amd import engine
    g = slim_eval_graph(with_cnn=False)
    p = _cut_prep(g)
    rng = np.random.default_rng(0)
    hw = np.concatenate([rng.integers(224, 900, (40, 2)), [[224, 224], [256, 1000], [1001, 257], [300, 300]]])
    got = p.row_params(hw.astype(np.int32))
    prog = engine.program(g.serialize(), ["new_h:0", "new_w:0", "off_h:0", "off_w:0"], ["DecodeJpeg"])
    for (H, W), row in zip(hw, got):
        img = torch.zeros((int(H), int(W), 3), dtype=torch.uint8)
        want = [int(t.item()) for t in engine.run_program(prog, [img], torch.device("cpu"))]
        assert list(row) == want, (H, W, row, want)


def _cut_prep(g):
    # the pre-stage of a graph whose cut is its `prepped` batch of one
    return core._match_image_prep(g.serialize(), ["DecodeJpeg"], "prepped", [1, 224, 224, 3])


def test_small_image_rows_fall_back():
    """A row whose central crop would fall outside its resize (the graph's
    own Slice would fail there) is not batched: the chunk runs per row."""
    p = _cut_prep(slim_eval_graph(side=200, with_cnn=False))
    with pytest.raises(image_prep.Unsupported):
        p.row_params(np.array([[300, 400]], np.int32))


def test_split_branches_with_different_steps_are_refused():
    g = tf.Graph()
    with g.as_default():
        data = tf.placeholder(tf.string, [], name="data")
        x = tf.cast(tf.image.decode_jpeg(data, channels=3, name="DecodeJpeg"), tf.float32)
        x = tf.slice(tf.squeeze(tf.image.resize_bilinear(tf.expand_dims(x, 0), [40, 40]), [0]), [4, 4, 0],
                     [32, 32, 3])
        r, gc, b = tf.split(x, 3, axis=2)
        x = tf.expand_dims(tf.concat([r - 1.0, gc * 2.0, b - 3.0], 2), 0, name="prepped")
    assert core._match_image_prep(g.serialize(), ["DecodeJpeg"], "prepped", [1, 32, 32, 3]) is None


def _shape_graph(variant):
    """decoded image -> a resize size / crop offset computed with the ops the
    host evaluator models (half-to-even Round, truncating and flooring
    integer division, Minimum / Maximum, Select, float64 arithmetic)"""
    g = tf.Graph()
    with g.as_default():
        data = tf.placeholder(tf.string, [], name="data")
        im = tf.image.decode_jpeg(data, channels=3, name="DecodeJpeg")
        s = tf.shape(im)
        h, w = s[0], s[1]
        if variant == "round_half_even":
            # x.5 cases: 0.5 * odd sizes
            nh = tf.cast(tf.round(tf.cast(h, tf.float32) * 0.5 + 40.0), tf.int32)
            nw = tf.cast(tf.round(tf.cast(w, tf.float32) * 0.5 + 40.0), tf.int32)
        elif variant == "float64_div":
            hd, wd = tf.cast(h, tf.float64), tf.cast(w, tf.float64)
            sc = 97.0 / tf.minimum(hd, wd)
            nh = tf.cast(hd * sc, tf.int32)
            nw = tf.cast(wd * sc, tf.int32)
        else:  # integer arithmetic with Maximum and FloorDiv / truncating Div
            nh = tf.maximum(h // 2, 64) + tf.floordiv(w - h, 7)
            nw = tf.maximum(w // 2, 64) + tf.div(h - w, 7)  # Div on int32: truncates toward zero
        nh = tf.identity(tf.maximum(nh, 64), name="new_h")
        nw = tf.identity(tf.maximum(nw, 64), name="new_w")
        x = tf.image.resize_bilinear(tf.expand_dims(im, 0), tf.stack([nh, nw]), align_corners=True)
        x = tf.squeeze(x, [0])
        oy = tf.identity((nh - 48) // 2, name="off_h")
        ox = tf.identity((nw - 48) // 2, name="off_w")
        x = tf.slice(x, tf.stack([oy, ox, 0]), [48, 48, 3])
        tf.expand_dims(x * (1.0 / 255.0), 0, name="prepped")
    return g


@pytest.mark.parametrize("variant", ["round_half_even", "float64_div", "int_ops"])
def test_shape_evaluator_matches_cpu_executor(variant):
    import torch

    from tensorframes_amd import engine
    g = _shape_graph(variant)
    p = core._match_image_prep(g.serialize(), ["DecodeJpeg"], "prepped", [1, 48, 48, 3])
    assert p is not None and p.dyn is not None and p.mode == 1
    rng = np.random.default_rng(3)
    hw = np.concatenate([rng.integers(60, 700, (30, 2)), [[61, 61], [63, 701], [99, 100], [301, 77]]]).astype(np.int32)
    try:
        got = p.row_params(hw)
    except image_prep.Unsupported:
        got = None
    prog = engine.program(g.serialize(), ["new_h:0", "new_w:0", "off_h:0", "off_w:0"], ["DecodeJpeg"])
    want = np.array([[int(t.item()) for t in engine.run_program(prog, [torch.zeros((int(H), int(W), 3), dtype=torch.uint8)],
                                                                  torch.device("cpu"))] for H, W in hw])
    if got is None:  # a row's crop falls outside its resize: the chunk runs per row
        assert np.any(want[:, 2] < 0) or np.any(want[:, 3] < 0) or np.any(want[:, 0] - want[:, 2] < 48)
    else:
        assert np.array_equal(got, want), (got[:4], want[:4])

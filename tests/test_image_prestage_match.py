"""The batched image pre-stage is recognised from the graph alone (CPU):
core._match_image_prep on the reference's JPEG scoring chain
(src/main/python/tensorframes_snippets/read_image.py:35-75: decode -> cast ->
resize -> central crop -> mean subtraction -> expand_dims) and on variants it
must take (channel count from the decoder) or refuse (ops it does not model)."""
import numpy as np

from tensorframes_amd import core, tf
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

"""Frozen CNN scoring graphs with random-init weights: Inception-v3 and VGG-16.

The reference scores images with frozen TF GraphDefs (VGG-16 via map_rows on a
binary JPEG column, reference: src/main/python/tensorframes_snippets/read_image.py:56-167;
BASELINE.json config 5 scores Inception-v3 with map_blocks). No checkpoints
can be downloaded here, so these builders emit the same architectures as
frozen inference GraphDefs (batch-norm folded into each conv's bias, NHWC,
TF op names: Conv2D / BiasAdd / Relu / MaxPool / AvgPool / ConcatV2 / Mean /
MatMul / Softmax) with random weights. The executor fuses every
Conv2D+BiasAdd+Relu into one implicit-GEMM MFMA kernel.

`width` scales every channel count (tests use small widths on the CPU).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from ..graph import dsl as tf


class _Builder:
    def __init__(self, seed: int, width: float, dtype=np.float32):
        self.rng = np.random.default_rng(seed)
        self.width = width
        self.dtype = dtype

    def ch(self, c: int) -> int:
        return max(1, int(round(c * self.width)))

    def conv(self, x, out_c: int, kh: int, kw: int, stride: int = 1, padding: str = "SAME",
             name: Optional[str] = None, relu: bool = True, scale_out: bool = True):
        in_c = x.get_shape().as_list()[-1]
        oc = self.ch(out_c) if scale_out else out_c
        with tf.name_scope(name or "conv"):
            std = np.sqrt(2.0 / (kh * kw * in_c))
            w = (self.rng.standard_normal((kh, kw, in_c, oc)) * std).astype(self.dtype)
            b = (self.rng.standard_normal(oc) * 0.01).astype(self.dtype)
            y = tf.nn.conv2d(x, tf.constant(w, name="weights"), [1, stride, stride, 1], padding)
            y = tf.nn.bias_add(y, tf.constant(b, name="biases"))
            return tf.nn.relu(y) if relu else y

    def fc(self, x, out: int, name: str, relu: bool):
        in_c = x.get_shape().as_list()[-1]
        with tf.name_scope(name):
            w = (self.rng.standard_normal((in_c, out)) * np.sqrt(2.0 / in_c)).astype(self.dtype)
            b = (self.rng.standard_normal(out) * 0.01).astype(self.dtype)
            y = tf.nn.bias_add(tf.matmul(x, tf.constant(w, name="weights")), tf.constant(b, name="biases"))
            return tf.nn.relu(y) if relu else y


def _max_pool(x, k, s, padding="VALID"):
    return tf.nn.max_pool(x, [1, k, k, 1], [1, s, s, 1], padding)


def _avg_pool(x, k, s, padding="SAME"):
    return tf.nn.avg_pool(x, [1, k, k, 1], [1, s, s, 1], padding)


def inception_v3(image_size: int = 299, num_classes: int = 1000, width: float = 1.0, seed: int = 0,
                 input_name: str = "image", output_name: str = "prob", graph: Optional[tf.Graph] = None,
                 inputs=None) -> Tuple[tf.Graph, str, str]:
    """Inception-v3 (Szegedy et al. 2015) as a frozen inference GraphDef.
    Global average pooling makes any input >= 75x75 valid (224x224 for the
    BASELINE config). Returns (graph, input placeholder name, output name);
    `inputs` (a [N,H,W,3] float32 tensor of `graph`) replaces the placeholder."""
    g = graph or (inputs.graph if inputs is not None else tf.Graph())
    B = _Builder(seed, width)
    with g.as_default():
        x = inputs if inputs is not None else tf.placeholder(tf.float32, [None, image_size, image_size, 3],
                                                             name=input_name)
        # stem
        y = B.conv(x, 32, 3, 3, 2, "VALID", "Conv2d_1a_3x3")
        y = B.conv(y, 32, 3, 3, 1, "VALID", "Conv2d_2a_3x3")
        y = B.conv(y, 64, 3, 3, 1, "SAME", "Conv2d_2b_3x3")
        y = _max_pool(y, 3, 2)
        y = B.conv(y, 80, 1, 1, 1, "VALID", "Conv2d_3b_1x1")
        y = B.conv(y, 192, 3, 3, 1, "VALID", "Conv2d_4a_3x3")
        y = _max_pool(y, 3, 2)

        def block_a(y, pool_c, name):
            with tf.name_scope(name):
                b0 = B.conv(y, 64, 1, 1, name="b0_1x1")
                b1 = B.conv(B.conv(y, 48, 1, 1, name="b1_1x1"), 64, 5, 5, name="b1_5x5")
                b2 = B.conv(B.conv(B.conv(y, 64, 1, 1, name="b2_1x1"), 96, 3, 3, name="b2_3x3a"),
                            96, 3, 3, name="b2_3x3b")
                b3 = B.conv(_avg_pool(y, 3, 1), pool_c, 1, 1, name="b3_1x1")
                return tf.concat([b0, b1, b2, b3], 3)

        y = block_a(y, 32, "Mixed_5b")
        y = block_a(y, 64, "Mixed_5c")
        y = block_a(y, 64, "Mixed_5d")
        with tf.name_scope("Mixed_6a"):
            b0 = B.conv(y, 384, 3, 3, 2, "VALID", name="b0_3x3")
            b1 = B.conv(B.conv(B.conv(y, 64, 1, 1, name="b1_1x1"), 96, 3, 3, name="b1_3x3"),
                        96, 3, 3, 2, "VALID", name="b1_3x3s2")
            y = tf.concat([b0, b1, _max_pool(y, 3, 2)], 3)

        def block_c(y, c7, name):
            with tf.name_scope(name):
                b0 = B.conv(y, 192, 1, 1, name="b0_1x1")
                b1 = B.conv(y, c7, 1, 1, name="b1_1x1")
                b1 = B.conv(b1, c7, 1, 7, name="b1_1x7")
                b1 = B.conv(b1, 192, 7, 1, name="b1_7x1")
                b2 = B.conv(y, c7, 1, 1, name="b2_1x1")
                b2 = B.conv(b2, c7, 7, 1, name="b2_7x1a")
                b2 = B.conv(b2, c7, 1, 7, name="b2_1x7a")
                b2 = B.conv(b2, c7, 7, 1, name="b2_7x1b")
                b2 = B.conv(b2, 192, 1, 7, name="b2_1x7b")
                b3 = B.conv(_avg_pool(y, 3, 1), 192, 1, 1, name="b3_1x1")
                return tf.concat([b0, b1, b2, b3], 3)

        y = block_c(y, 128, "Mixed_6b")
        y = block_c(y, 160, "Mixed_6c")
        y = block_c(y, 160, "Mixed_6d")
        y = block_c(y, 192, "Mixed_6e")
        with tf.name_scope("Mixed_7a"):
            b0 = B.conv(B.conv(y, 192, 1, 1, name="b0_1x1"), 320, 3, 3, 2, "VALID", name="b0_3x3")
            b1 = B.conv(y, 192, 1, 1, name="b1_1x1")
            b1 = B.conv(b1, 192, 1, 7, name="b1_1x7")
            b1 = B.conv(b1, 192, 7, 1, name="b1_7x1")
            b1 = B.conv(b1, 192, 3, 3, 2, "VALID", name="b1_3x3")
            y = tf.concat([b0, b1, _max_pool(y, 3, 2)], 3)

        def block_e(y, name):
            with tf.name_scope(name):
                b0 = B.conv(y, 320, 1, 1, name="b0_1x1")
                b1 = B.conv(y, 384, 1, 1, name="b1_1x1")
                b1 = tf.concat([B.conv(b1, 384, 1, 3, name="b1_1x3"), B.conv(b1, 384, 3, 1, name="b1_3x1")], 3)
                b2 = B.conv(B.conv(y, 448, 1, 1, name="b2_1x1"), 384, 3, 3, name="b2_3x3")
                b2 = tf.concat([B.conv(b2, 384, 1, 3, name="b2_1x3"), B.conv(b2, 384, 3, 1, name="b2_3x1")], 3)
                b3 = B.conv(_avg_pool(y, 3, 1), 192, 1, 1, name="b3_1x1")
                return tf.concat([b0, b1, b2, b3], 3)

        y = block_e(y, "Mixed_7b")
        y = block_e(y, "Mixed_7c")
        y = tf.reduce_mean(y, [1, 2], name="global_pool")
        logits = B.fc(y, num_classes, "Logits", relu=False)
        tf.nn.softmax(logits, name=output_name)
    return g, input_name, output_name


def vgg16(image_size: int = 224, num_classes: int = 1000, width: float = 1.0, fc_width: int = 4096,
          seed: int = 0, input_name: str = "image", output_name: str = "prob",
          graph: Optional[tf.Graph] = None, inputs=None) -> Tuple[tf.Graph, str, str]:
    """VGG-16 (Simonyan & Zisserman 2014) as a frozen GraphDef (the network of
    the reference's read_image.py)."""
    g = graph or (inputs.graph if inputs is not None else tf.Graph())
    B = _Builder(seed, width)
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    with g.as_default():
        x = inputs if inputs is not None else tf.placeholder(tf.float32, [None, image_size, image_size, 3],
                                                             name=input_name)
        y = x
        i = 0
        for c in cfg:
            if c == "M":
                y = _max_pool(y, 2, 2)
            else:
                i += 1
                y = B.conv(y, c, 3, 3, 1, "SAME", f"conv{i}")
        shp = y.get_shape().as_list()
        y = tf.reshape(y, [-1, shp[1] * shp[2] * shp[3]])
        y = B.fc(y, fc_width, "fc6", relu=True)
        y = B.fc(y, fc_width, "fc7", relu=True)
        logits = B.fc(y, num_classes, "fc8", relu=False)
        tf.nn.softmax(logits, name=output_name)
    return g, input_name, output_name


def top_k_classes(graph: tf.Graph, output_name: str = "prob", k: int = 5, name: str = "top"):
    """Adds `TopKV2` on the class probabilities (reference: read_image.py:71)."""
    with graph.as_default():
        prob = graph.get_tensor_by_name(output_name + ":0")
        vals, idx = tf.nn.top_k(prob, k, name=name)
        return tf.identity(vals, name=name + "_values"), tf.identity(idx, name=name + "_indices")


# ImageNet channel means (RGB, 0-255 scale), as in VGG preprocessing
_RGB_MEANS = np.array([123.68, 116.78, 103.94], np.float32)


def slim_eval_preprocess(im, image_size: int = 224, resize_side: int = 256):
    """The slim-style eval preprocessing (vgg_preprocessing.preprocess_for_eval,
    the graphs the reference's users score with): aspect-preserving bilinear
    resize of the uint8 image so its smaller side is `resize_side` (sizes
    computed from the image's own shape, rounded half to even), a central
    `image_size` crop whose offsets come from the resized shape, float, and the
    per-channel mean subtracted channel by channel (split / concat)."""
    shp = tf.shape(im)
    hf, wf = tf.cast(shp[0], tf.float32), tf.cast(shp[1], tf.float32)
    scale = tf.where(tf.greater(hf, wf), float(resize_side) / wf, float(resize_side) / hf)
    nh = tf.cast(tf.round(hf * scale), tf.int32)
    nw = tf.cast(tf.round(wf * scale), tf.int32)
    x = tf.squeeze(tf.image.resize_bilinear(tf.expand_dims(im, 0), [nh, nw]), [0])
    rs = tf.shape(x)
    oy, ox = (rs[0] - image_size) // 2, (rs[1] - image_size) // 2
    x = tf.cast(tf.slice(x, [oy, ox, 0], [image_size, image_size, 3]), tf.float32)
    chans = tf.split(x, 3, axis=2)
    return tf.concat([c - m for c, m in zip(chans, _RGB_MEANS)], 2)


def jpeg_scoring_graph(model: str = "vgg16", image_size: int = 224, resize_to: Optional[int] = None,
                       contents=None, k: int = 5, preprocessing: str = "reference", **model_kw) -> tf.Graph:
    """The reference's image-scoring graph (read_image.py:35-75): JPEG bytes ->
    ``DecodeJpeg`` (host stage) -> float -> resize -> central crop -> mean
    subtraction -> batch of one -> CNN -> softmax -> ``top_predictions``
    (TopKV2). `contents` (bytes) becomes the ``DecodeJpeg/contents`` constant
    that ``map_rows(..., feed_dict={'DecodeJpeg/contents': <binary column>})``
    replaces row by row; None makes it a string placeholder of that name.
    preprocessing="slim": slim_eval_preprocess (aspect-preserving resize to
    `resize_to`, default 256) instead of the square resize.
    Outputs: ``index`` (int32 [k]) and ``value`` (float32 [k])."""
    g = tf.Graph()
    resize_to = resize_to or image_size + 32
    with g.as_default():
        if contents is None:
            with tf.name_scope("DecodeJpeg/"):
                contents = tf.placeholder(tf.string, [], name="contents")
        im = tf.image.decode_jpeg(contents, channels=3)
        if preprocessing == "slim":
            x = slim_eval_preprocess(im, image_size, resize_to)
        else:
            x = tf.cast(im, tf.float32)
            x = tf.image.resize_images(x, [resize_to, resize_to])
            x = tf.image.central_crop_to(x, image_size, image_size)
            x = tf.subtract(x, tf.constant(_RGB_MEANS))
        x = tf.expand_dims(x, 0)
        build = {"vgg16": vgg16, "inception_v3": inception_v3}[model]
        build(image_size=image_size, inputs=x, graph=g, **model_kw)
        prob = g.get_tensor_by_name("prob:0")
        vals, idx = tf.nn.top_k(tf.squeeze(prob), k, name="top_predictions")
        tf.identity(idx, name="index")
        tf.identity(vals, name="value")
    return g

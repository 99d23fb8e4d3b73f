"""The batched image pre-stage of map_rows image scoring (core._ImagePrep,
kernels/image.hip ragged_prep_kernel): the reference's JPEG scoring graph
(src/main/python/tensorframes_snippets/read_image.py:35-75, one image per row)
run with the per-row pre-program and with the ragged-batch kernel must give
bit-identical top-k values and indices; the kernel alone against the per-image
CPU-oracle ops (Cast -> ResizeBilinear -> Slice -> Sub) on images of mixed
sizes and every resize mode; the slim-style eval preprocessing (aspect-preserving
resize computed from each image's shape, central crop, per-channel mean
through split/concat) against the CPU executor, bit for bit."""
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import Row, engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402
from tensorframes_amd.models import cnn  # noqa: E402

DEV = torch.device("cuda", 0)


def _jpegs(n, rng):
    from PIL import Image
    out = []
    for _ in range(n):
        h, w = rng.integers(60, 160, 2)
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(buf, format="JPEG", quality=90)
        out.append(bytearray(buf.getvalue()))
    return out


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_ragged_kernel_matches_per_image_ops(mode):
    rng = np.random.default_rng(mode)
    imgs = [rng.integers(0, 255, (int(h), int(w), 3), dtype=np.uint8) for h, w in rng.integers(20, 90, (7, 2))]
    OH, OW, oy, ox, h, w = 48, 40, 4, 3, 40, 33
    mean = [10.5, -3.25, 100.0]
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.uint8, [None, None, 3], name="x")
        y = tf.cast(x, tf.float32)
        y = tf.image.resize_bilinear(tf.expand_dims(y, 0), [OH, OW], align_corners=mode == 1,
                                     half_pixel_centers=mode == 2)
        y = tf.slice(tf.squeeze(y, [0]), [oy, ox, 0], [h, w, -1])
        tf.multiply(tf.subtract(y, tf.constant(np.array(mean, np.float32))), 0.5, name="out")
    prog = engine.program(g.serialize(), ["out"], ["x"])
    # the oracle is the CPU executor; the GPU per-row program gives the same bits
    want = [engine.run_program(prog, [torch.from_numpy(a)], torch.device("cpu"))[0] for a in imgs]
    for a, wnt in zip(imgs[:3], want):
        assert torch.equal(engine.run_program(prog, [torch.from_numpy(a)], DEV)[0].cpu(), wnt)
    sizes = np.array([a.size for a in imgs])
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)).to(DEV)
    hw = torch.tensor([[a.shape[0], a.shape[1]] for a in imgs], dtype=torch.int32, device=DEV)
    data = torch.from_numpy(np.concatenate([a.reshape(-1) for a in imgs])).to(DEV)
    got = _C.ragged_image_prep(data, offs, hw, 3, OH, OW, mode, oy, ox, h, w, [(1, mean), (2, [0.5])]).cpu()
    assert got.shape == (len(imgs), h, w, 3)
    for i, wnt in enumerate(want):
        assert torch.equal(got[i], wnt), f"image {i}: max diff {(got[i] - wnt).abs().max().item()}"


@pytest.mark.parametrize("native", [False, True])
def test_batched_prestage_equals_per_row_scoring(native):
    rng = np.random.default_rng(5)
    jpgs = _jpegs(70, rng)
    # a grayscale file among the RGB ones (DecodeJpeg channels=3 replicates it)
    buf = io.BytesIO()
    from PIL import Image
    Image.fromarray(rng.integers(0, 255, (90, 120), dtype=np.uint8)).save(buf, format="JPEG")
    jpgs[17] = bytearray(buf.getvalue())
    df = tfs.create_dataframe([Row(uri=f"img{i}", image_data=b) for i, b in enumerate(jpgs)], num_partitions=1)
    g = cnn.jpeg_scoring_graph("vgg16", contents=bytes(jpgs[0]), width=0.125)
    res = {}
    try:
        for on in (False, True):
            tfs.set_config(map_rows_batched_prestage=on, native_jpeg_decode=native)
            tfs.metrics.reset()
            with g.as_default():
                pred = tfs.map_rows(["index", "value"], df, feed_dict={"DecodeJpeg/contents": "image_data"})
                rows = pred.select("uri", "index", "value").collect()
            res[on] = rows
            m = tfs.metrics.snapshot()
            assert (m.get("map_rows_batched_prestage_rows", 0) == len(jpgs)) == on
            assert (m.get("map_rows_native_decode_rows", 0) == len(jpgs)) == (on and native)
    finally:
        tfs.set_config(map_rows_batched_prestage=True, native_jpeg_decode=True)
    for a, b in zip(res[False], res[True]):
        assert a.uri == b.uri
        assert list(a["index"]) == list(b["index"])
        assert np.array_equal(np.asarray(a["value"]), np.asarray(b["value"]))


def test_unknown_libjpeg_version_falls_back_with_identical_topk():
    """The loaded libjpeg seen as an unknown version (jpeg_force_version): the
    pre-stage refuses the native decoder (jpeg_native_unavailable), decodes
    through the Python decoder and gives the native run's top-k bit for bit."""
    from tensorframes_amd import core
    rng = np.random.default_rng(6)
    jpgs = _jpegs(40, rng)
    df = tfs.create_dataframe([Row(uri=f"img{i}", image_data=b) for i, b in enumerate(jpgs)], num_partitions=1)
    g = cnn.jpeg_scoring_graph("vgg16", contents=bytes(jpgs[0]), width=0.125)
    res, snaps = {}, {}
    try:
        for forced in (0, 99):
            _C.jpeg_force_version(forced)
            tfs.metrics.reset()
            with g.as_default():
                pred = tfs.map_rows(["index", "value"], df, feed_dict={"DecodeJpeg/contents": "image_data"})
                res[forced] = pred.select("uri", "index", "value").collect()
            snaps[forced] = tfs.metrics.snapshot()
    finally:
        _C.jpeg_force_version(0)
        core._JPEG_CHECKED.clear()
    assert snaps[0].get("map_rows_native_decode_rows", 0) == len(jpgs)
    assert snaps[99].get("map_rows_native_decode_rows", 0) == 0
    assert snaps[99].get("jpeg_native_unavailable", 0) >= 1
    assert snaps[99].get("map_rows_batched_prestage_rows", 0) == len(jpgs)
    for a, b in zip(res[0], res[99]):
        assert a.uri == b.uri
        assert list(a["index"]) == list(b["index"])
        assert np.array_equal(np.asarray(a["value"]), np.asarray(b["value"]))


def test_native_decode_falls_back_for_truncated_files():
    """A truncated JPEG in a chunk: the native decoder reports it, the Python
    decoder then raises its own error, as on the per-row path."""
    rng = np.random.default_rng(9)
    jpgs = _jpegs(8, rng)
    jpgs[3] = jpgs[3][:len(jpgs[3]) // 2]
    df = tfs.create_dataframe([Row(image_data=b) for b in jpgs], num_partitions=1)
    g = cnn.jpeg_scoring_graph("vgg16", contents=bytes(jpgs[0]), width=0.125)
    with g.as_default(), pytest.raises(Exception, match="(?i)truncated"):
        tfs.map_rows(["index", "value"], df, feed_dict={"DecodeJpeg/contents": "image_data"}).collect()


def _slim_graph(**kw):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_image_prestage_match import slim_eval_graph
    return slim_eval_graph(**kw)


def test_slim_prestage_equals_cpu_executor():
    """Per-row resize sizes and crop offsets (from each image's own shape)
    through the ragged kernel: bit-identical to the CPU executor running the
    graph's pre-part on each image."""
    from tensorframes_amd import core
    g = _slim_graph(with_cnn=False)
    prep = core._match_image_prep(g.serialize(), ["DecodeJpeg"], "prepped", [1, 224, 224, 3])
    assert prep is not None and prep.dyn is not None
    rng = np.random.default_rng(4)
    shapes = [(224, 224), (256, 300), (480, 270), (231, 999), (640, 480), (225, 227)]
    imgs = [rng.integers(0, 255, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    got = prep.run(imgs, DEV).cpu()
    prog = engine.program(g.serialize(), ["prepped:0"], ["DecodeJpeg"])
    for i, a in enumerate(imgs):
        want = engine.run_program(prog, [torch.from_numpy(a)], torch.device("cpu"))[0]
        assert want.shape == (1, 224, 224, 3)
        assert torch.equal(got[i:i + 1], want), f"image {shapes[i]}: max diff {(got[i] - want[0]).abs().max().item()}"


@pytest.mark.parametrize("native", [False, True])
def test_slim_scoring_batched_equals_per_row(native):
    """The slim-style graph through map_rows: the batched pre-stage runs
    (metric counters) and gives the per-row path's top-k bit for bit."""
    from PIL import Image
    rng = np.random.default_rng(8)
    jpgs = []
    for _ in range(24):
        h, w = (int(v) for v in rng.integers(224, 400, 2))
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(buf, format="JPEG", quality=90)
        jpgs.append(bytearray(buf.getvalue()))
    df = tfs.create_dataframe([Row(uri=f"img{i}", image_data=b) for i, b in enumerate(jpgs)], num_partitions=1)
    g = _slim_graph()
    res = {}
    try:
        for on in (False, True):
            tfs.set_config(map_rows_batched_prestage=on, native_jpeg_decode=native)
            tfs.metrics.reset()
            with g.as_default():
                rows = tfs.map_rows(["s"], df, feed_dict={"data": "image_data"}).select("uri", "s").collect()
            res[on] = rows
            m = tfs.metrics.snapshot()
            assert (m.get("map_rows_batched_prestage_rows", 0) == len(jpgs)) == on, m
            assert (m.get("map_rows_prestage_row_params_rows", 0) == len(jpgs)) == on, m
    finally:
        tfs.set_config(map_rows_batched_prestage=True, native_jpeg_decode=True)
    for a, b in zip(res[False], res[True]):
        assert a.uri == b.uri
        assert np.array_equal(np.asarray(a["s"]), np.asarray(b["s"]))


@pytest.mark.parametrize("variant", ["round_half_even", "float64_div", "int_ops"])
def test_per_row_align_corners_and_shape_ops_equal_cpu_executor(variant):
    """Per-row sizes from the host shape evaluator, align_corners resize,
    a scale step: the ragged kernel against the CPU executor, bit for bit."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_image_prestage_match import _shape_graph

    from tensorframes_amd import core
    g = _shape_graph(variant)
    prep = core._match_image_prep(g.serialize(), ["DecodeJpeg"], "prepped", [1, 48, 48, 3])
    assert prep is not None and prep.dyn is not None
    rng = np.random.default_rng(11)
    shapes = [(120, 160), (97, 301), (250, 99), (64, 64), (333, 222)]
    imgs = [rng.integers(0, 255, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    got = prep.run(imgs, DEV)
    assert got is not None
    got = got.cpu()
    prog = engine.program(g.serialize(), ["prepped:0"], ["DecodeJpeg"])
    for i, a in enumerate(imgs):
        want = engine.run_program(prog, [torch.from_numpy(a)], torch.device("cpu"))[0]
        assert torch.equal(got[i:i + 1], want), f"{shapes[i]}: max diff {(got[i] - want[0]).abs().max().item()}"

"""Native JPEG decode (csrc/runtime/jpeg_decode.cpp): libjpeg through dlopen on
a GIL-free thread pool, decoding a chunk of cells straight into the ragged
[offsets | hw | pixels] buffer of the batched image pre-stage. Its pixels must
equal the Python decoder's (ops/host_ops.decode_image, PIL) bit for bit on
baseline, progressive, grayscale and chroma-subsampled files; images it
cannot take are reported, not guessed. The reference decodes in
libtensorflow's DecodeJpeg (src/main/python/tensorframes_snippets/read_image.py:42)."""
import io

import numpy as np
import pytest

from tensorframes_amd._native import _C
from tensorframes_amd.ops.host_ops import decode_image

PIL = pytest.importorskip("PIL.Image")

if not _C.jpeg_native_available()[0]:
    pytest.skip(f"native JPEG decode unavailable: {_C.jpeg_native_available()[1]}", allow_module_level=True)


def _jpegs(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        i = len(out)
        h, w = (int(v) for v in rng.integers(9, 260, 2))
        if i % 4 == 0:  # smooth content
            a = np.repeat(np.linspace(0, 255, w)[None, :, None], h, 0).repeat(3, 2).astype(np.uint8)
        else:
            a = rng.integers(0, 255, (h, w, 3), dtype=np.uint8)
        im = PIL.fromarray(a)
        if i % 5 == 0:
            im = im.convert("L")
        kw = {"quality": int(rng.integers(30, 100))}
        if i % 3 == 0:
            kw["progressive"] = True
        if i % 2 == 0:
            kw["subsampling"] = int(rng.integers(0, 3))
        buf = io.BytesIO()
        try:
            im.save(buf, format="JPEG", **kw)
        except OSError:  # some encoder settings refuse tiny progressive images
            continue
        out.append(bytearray(buf.getvalue()))
    return out


def test_single_decode_matches_pil():
    for d in _jpegs(60):
        want = decode_image(d, 3)
        got = _C.jpeg_decode(d, 3).numpy()
        assert got.shape == want.shape
        assert np.array_equal(got, want)


def test_grayscale_to_one_channel():
    buf = io.BytesIO()
    PIL.fromarray(np.arange(64 * 48, dtype=np.uint8).reshape(48, 64) * 3).save(buf, format="JPEG")
    got = _C.jpeg_decode(buf.getvalue(), 1).numpy()
    assert np.array_equal(got, decode_image(buf.getvalue(), 1))


@pytest.mark.parametrize("threads", [1, 4])
def test_batch_layout_matches_pil(threads):
    cells = _jpegs(40, seed=threads)
    job = _C.JpegBatch(cells, 3, threads, False)
    assert job.header_ok
    assert job.wait() == []
    hb = job.buffer.numpy()
    n = len(cells)
    offs = hb[:8 * n].view(np.int64)
    hw = hb[8 * n:job.meta_bytes].view(np.int32).reshape(n, 2)
    assert job.offsets_bytes == 8 * n and job.meta_bytes == 16 * n
    for i, c in enumerate(cells):
        want = decode_image(c, 3)
        assert tuple(hw[i]) == want.shape[:2] and offs[i] == job.pixel_offset(i)
        o = job.meta_bytes + offs[i]
        assert np.array_equal(hb[o:o + want.size].reshape(want.shape), want)


def test_truncated_image_is_reported_not_guessed():
    cells = _jpegs(3, seed=7)
    cells[1] = cells[1][:len(cells[1]) // 2]
    job = _C.JpegBatch(cells, 3, 2, False)
    assert job.header_ok
    assert job.wait() == [1]


def test_non_jpeg_cells_fail_the_header_pass():
    buf = io.BytesIO()
    PIL.fromarray(np.zeros((8, 8, 3), np.uint8)).save(buf, format="PNG")
    cells = _jpegs(2) + [bytearray(buf.getvalue())]
    job = _C.JpegBatch(cells, 3, 2, False)
    assert not job.header_ok and job.bad_header == 2
    with pytest.raises(Exception):
        _C.jpeg_decode(buf.getvalue(), 3)


def test_concurrent_batches_share_the_pool():
    """Several batches in flight at once (the pre-stage keeps the next chunk
    decoding while the current one is consumed) all complete, each into its
    own buffer."""
    cells = _jpegs(24, seed=11)
    jobs = [_C.JpegBatch(cells[i::3], 3, 4, False) for i in range(3)]
    for i, job in enumerate(jobs):
        assert job.wait() == []
        hb = job.buffer.numpy()
        for j, c in enumerate(cells[i::3]):
            want = decode_image(c, 3)
            o = job.meta_bytes + job.pixel_offset(j)
            assert np.array_equal(hb[o:o + want.size].reshape(want.shape), want)


def test_batch_outlives_dropped_job():
    """A JpegBatch dropped before wait() must not leave tasks writing into
    freed memory: the destructor waits for its tasks."""
    cells = _jpegs(16, seed=12)
    for _ in range(5):
        job = _C.JpegBatch(cells, 3, 4, False)
        del job
    assert _C.decode_pool_threads() >= 1

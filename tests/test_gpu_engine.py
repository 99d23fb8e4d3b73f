"""GPU engine paths: pipelined host->HBM->host chunk loop, device-resident
frames, pinned pool, monoid reductions, segmented aggregate."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import engine, tf  # noqa: E402
from tensorframes_amd._native import _C  # noqa: E402

rng = np.random.default_rng(7)


def test_pinned_pool_is_pinned_and_reused():
    a = _C.empty_pinned([1 << 20], torch.float32)
    assert _C.is_pinned(a)
    assert not _C.is_pinned(torch.empty(1 << 20))
    p = a.data_ptr()
    del a
    b = _C.empty_pinned([1 << 20], torch.float32)
    assert b.data_ptr() == p  # came back from the pool


@pytest.mark.parametrize("rows", [70000, 300001])
def test_map_blocks_pipelined_matches_reference(rows):
    x = rng.standard_normal((rows, 64)).astype(np.float32)
    w = rng.standard_normal((64, 48)).astype(np.float32)
    df = tfs.analyze(tfs.from_columns({"x": x}, num_partitions=3, pinned=True))
    tfs.set_config(chunk_bytes=64 * 1024 * 10, min_chunked_rows=1000)
    try:
        with tf.Graph().as_default():
            xb = tfs.block(df, "x")
            y = tf.nn.relu(tf.matmul(xb, tf.constant(w)) + 1.0, name="y")
            z = tf.reduce_sum(xb * xb, [1], name="z")
            out = tfs.map_blocks([y, z], df)
            got_y, got_z = out.to_numpy("y"), out.to_numpy("z")
    finally:
        tfs.set_config(chunk_bytes=128 << 20, min_chunked_rows=65536)
    np.testing.assert_allclose(got_y, np.maximum(x.astype(np.float64) @ w + 1.0, 0), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(got_z, (x.astype(np.float64) ** 2).sum(1), rtol=1e-5, atol=1e-3)


def test_device_resident_frame_stays_on_device():
    x = rng.standard_normal((5000, 16)).astype(np.float64)
    df = tfs.from_columns({"x": x}, num_partitions=2).cache_on_device()
    with tf.Graph().as_default():
        xb = tf.placeholder(tf.float64, [None, None], name="x")
        y = tf.add(xb, 2.0, name="y")
        out = tfs.map_blocks(y, df)
        blocks = out.local_blocks()
    assert all(b.columns["y"].is_cuda for b in blocks.values())
    np.testing.assert_allclose(out.to_numpy("y"), x + 2.0)


def test_reduce_blocks_monoid_on_gpu():
    x = rng.standard_normal((100000, 1024)).astype(np.float32)
    df = tfs.analyze(tfs.from_columns({"x": x}, num_partitions=8))
    with tf.Graph().as_default():
        xi = tf.placeholder(tf.float32, [None, 1024], name="x_input")
        s = tf.reduce_sum(xi, [0], name="x")
        got = tfs.reduce_blocks(s, df)
    np.testing.assert_allclose(got, x.astype(np.float64).sum(0), rtol=1e-4, atol=1e-2)


def test_aggregate_segment_reduce_gpu():
    n = 20000
    keys = rng.integers(0, 50, n)
    x = rng.standard_normal((n, 8))
    df = tfs.create_dataframe([tfs.Row(key=int(k), x=list(v)) for k, v in zip(keys, x)])
    df = tfs.analyze(df)
    with tf.Graph().as_default():
        xi = tfs.block(df, "x", tf_name="x_input")
        s = tf.reduce_sum(xi, [0], name="x")
        rows = tfs.aggregate(s, df.groupBy("key")).collect()
    assert len(rows) == 50
    for r in rows:
        np.testing.assert_allclose(r.x, x[keys == r.key].sum(0), rtol=1e-10, atol=1e-9)


def test_hip_graph_replay_matches_eager_and_outputs_do_not_alias():
    """After a few warm runs a small plan is captured into a HIP graph and
    replayed; every replay must equal the eager result, and earlier outputs
    must not be overwritten by later replays."""
    import numpy as np
    from tensorframes_amd import engine, tf
    g = tf.Graph()
    rng = np.random.default_rng(3)
    w = rng.standard_normal((64, 32)).astype(np.float32)
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 64], name="x")
        # enough kernels for capture to pay off (kGraphMinSteps)
        for i in range(16):
            x = tf.nn.relu(tf.matmul(x, tf.constant(rng.standard_normal((64, 64)).astype(np.float32) / 8)))
        h = tf.nn.relu(tf.matmul(x, tf.constant(w)))
        y = tf.reduce_sum(tf.square(h - 1.0), [1], name="y")
        tf.nn.softmax(h * 0.1, name="p")
    prog = engine.program(g.serialize(), ["y", "p"], ["x"])
    dev = torch.device("cuda", 0)
    outs, refs = [], []
    for i in range(8):
        xin = torch.randn((256, 64), generator=torch.Generator().manual_seed(i))
        outs.append(engine.run_program(prog, [xin.to(dev)], dev))
        refs.append(engine.run_program(prog, [xin], torch.device("cpu")))
    torch.cuda.synchronize()
    st = prog.stats()
    assert st["graphs_captured"] >= 1 and st["graph_replays"] >= 4 and st["graph_failures"] == 0
    for o, r in zip(outs, refs):
        for a, b in zip(o, r):
            torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-4)


def test_zero_copy_replay_for_device_inputs_at_stable_addresses():
    """Device inputs that come back at the same addresses (the partitions of a
    device-cached frame, run every iteration) are captured on the caller's own
    tensors and replayed with no input copy: the replay must read the CURRENT
    contents of those tensors (updated in place between runs), outputs of
    earlier runs must stay intact, and a 20 MB input is no obstacle."""
    import numpy as np
    from tensorframes_amd import engine, tf
    rng = np.random.default_rng(4)
    c = rng.standard_normal((10, 100))
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, [None, 100], name="x")
        d = tf.reduce_sum(tf.square(x), [1], keep_dims=True) - 2 * tf.matmul(x, tf.constant(c), transpose_b=True)
        idx = tf.argmin(d, 1, name="i")
        tf.reduce_min(d, [1], name="m")
        # the K-Means per-cluster sums: a few more kernels (>= 4 steps)
        tf.unsorted_segment_sum(x, idx, 10, name="s")
        tf.reduce_sum(tf.unsorted_segment_sum(tf.ones_like(d), idx, 10), [1], name="n")
    prog = engine.program(g.serialize(), ["i", "m", "s", "n"], ["x"])
    dev = torch.device("cuda", 0)
    parts = [torch.randn((25000, 100), dtype=torch.float64, device=dev) for _ in range(2)]
    before = prog.stats()
    outs = []
    for it in range(6):
        for p in parts:
            p.mul_(1.01)  # in place: same address, new values
            outs.append((engine.run_program(prog, [p], dev), p.cpu().numpy().copy()))
    torch.cuda.synchronize()
    st = prog.stats()
    # every output is kept alive here: after the first replay (outputs are
    # aliases of the graph's buffers) each address gets a second, cloning
    # instance whose replays copy their outputs out
    assert st["graphs_captured"] - before["graphs_captured"] == 4
    assert st["graph_replays"] - before["graph_replays"] >= 6
    assert st["graph_busy"] - before["graph_busy"] >= 4
    for (i, m, sm, n), xin in outs:
        dd = (xin ** 2).sum(1, keepdims=True) - 2 * xin @ c.T
        want_i = dd.argmin(1)
        np.testing.assert_array_equal(i.cpu().numpy(), want_i)
        np.testing.assert_allclose(m.cpu().numpy(), dd.min(1), rtol=1e-9, atol=1e-9)
        want_s = np.zeros((10, 100))
        np.add.at(want_s, want_i, xin)
        np.testing.assert_allclose(sm.cpu().numpy(), want_s, rtol=1e-9, atol=1e-8)
        np.testing.assert_allclose(n.cpu().numpy(), np.bincount(want_i, minlength=10) * 10.0)


def test_pipeline_stage_device_timers():
    """run_chunked brackets every chunk's H2D, compute and D2H with hipEvent
    pairs: the stage device times are positive, each below the wall time of
    the call, and exported as metrics for this call only."""
    import numpy as np
    from tensorframes_amd import engine, tf
    from tensorframes_amd.utils.logging import metrics
    g = tf.Graph()
    w = np.random.default_rng(4).standard_normal((256, 256)).astype(np.float32)
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 256], name="x")
        tf.nn.relu(tf.matmul(x, tf.constant(w)), name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    xin = torch.randn((400_000, 256))
    m0 = metrics.snapshot()
    out = engine.run_segments_pipelined(prog, [[xin]], [[((400_000, 256), torch.float32)]])
    m1 = metrics.snapshot()
    st = prog.stats()
    assert st["chunks"] >= 2
    for k in ("h2d_ms", "compute_ms", "d2h_ms"):
        assert 0 < st[k] < st["wall_ms"], (k, st)
        key = "pipeline_" + k.replace("_ms", "_device_ms")
        assert abs((m1.get(key, 0) - m0.get(key, 0)) - st[k]) < 1e-6
    assert m1["chunks"] - m0.get("chunks", 0) == st["chunks"]
    torch.testing.assert_close(out[0][0][:100], torch.relu(xin[:100] @ torch.as_tensor(w)), rtol=1e-4, atol=1e-4)


def test_concat_write_into_slice_matches_cpu():
    """Inception-style block: conv branches (+bias+relu) concatenated on the
    channel axis write straight into the concat output, and so does the
    pooled branch (planner-fused pool); a reused branch is copied. Result
    must equal the CPU executor."""
    import numpy as np
    from tensorframes_amd import engine, tf
    r = np.random.default_rng(9)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 9, 9, 16], name="x")

        def conv(t, oc, k):
            w = tf.constant((r.standard_normal((k, k, t.get_shape().as_list()[-1], oc)) * 0.1).astype(np.float32))
            b = tf.constant(r.standard_normal(oc).astype(np.float32))
            return tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(t, w, [1, 1, 1, 1], "SAME"), b))
        a = conv(x, 12, 1)
        b = conv(conv(x, 8, 1), 20, 3)
        shared = conv(x, 4, 1)
        p = tf.nn.avg_pool(x, [1, 3, 3, 1], [1, 1, 1, 1], "SAME")
        cat = tf.concat([a, b, p, shared], 3)
        tf.identity(cat, name="y")
        tf.identity(shared * 2.0, name="z")  # `shared` has two consumers: not aliased
    prog = engine.program(g.serialize(), ["y", "z"], ["x"])
    x_ = torch.randn((3, 9, 9, 16))
    dev = torch.device("cuda", 0)
    plan = prog.describe([x_.to(dev)])
    assert plan.count("->concat-slice@") == 3 and "(3 inputs written in place)" in plan
    gpu = engine.run_program(prog, [x_.to(dev)], dev)
    cpu = engine.run_program(prog, [x_], torch.device("cpu"))
    for a_, b_ in zip(gpu, cpu):
        torch.testing.assert_close(a_.cpu(), b_, rtol=1e-4, atol=1e-4)


def test_reduce_blocks_streams_large_host_partitions():
    """A host partition larger than the staging budget is reduced chunk by
    chunk on the GPU and the partials folded by the same graph."""
    import numpy as np
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.utils.logging import metrics
    x = np.random.default_rng(4).standard_normal((400_000, 64)).astype(np.float32)
    df = tfs.from_columns({"x": x}, num_partitions=1)
    old = tfs.config.chunk_bytes
    tfs.set_config(chunk_bytes=1 << 17)
    try:
        before = metrics.snapshot().get("reduce_blocks_chunks", 0)
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.float32, [None, 64], name="x_input")
            s, mx = tfs.reduce_blocks([tf.reduce_sum(xi, [0], name="x")], df), None
        assert metrics.snapshot().get("reduce_blocks_chunks", 0) - before >= 3
    finally:
        tfs.set_config(chunk_bytes=old)
    np.testing.assert_allclose(s, x.astype(np.float64).sum(0), rtol=1e-4, atol=1e-2)


def test_const_upload_is_async_and_ordered_across_streams():
    """A new program's constants go up asynchronously on the stream of its
    first run; a run on another stream waits for that copy (executor.cpp
    upload_consts / wait_consts)."""
    rng = np.random.default_rng(0)
    w = rng.standard_normal((256, 256)).astype(np.float32)
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.float32, [None, 256], name="x")
        tf.matmul(x, tf.constant(w), name="y")
    prog = engine.program(g.serialize(), ["y"], ["x"])
    dev = torch.device("cuda", 0)
    xin = torch.randn(4096, 256, device=dev)
    big = torch.randn(4096, 4096, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(8):  # keep the side stream busy so its upload lands late
            big = torch.mm(big, big) * 1e-3
        y1 = engine.run_program(prog, [xin], dev)[0]
    y2 = engine.run_program(prog, [xin], dev)[0]  # default stream: ordered after side's upload
    torch.cuda.synchronize()
    ref = (xin.double() @ torch.from_numpy(w).double().to(dev)).float()
    assert torch.allclose(y1, ref, atol=1e-3, rtol=1e-4)
    assert torch.allclose(y2, ref, atol=1e-3, rtol=1e-4)


def test_cat_rows_batched_copy_matches_torch_cat():
    """engine.cat_rows of many small device pieces (one batched-copy kernel,
    kernels/extra.hip): equal to torch.cat, for aligned, unaligned, empty and
    strided pieces, and above the 32-piece launch batch."""
    from tensorframes_amd import engine
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for dt in (torch.float64, torch.float32, torch.int32, torch.uint8):
        for trail in ((), (3,), (10, 100)):
            pieces = [torch.randint(0, 100, (n,) + trail, device=dev, generator=g).to(dt) for n in
                      [1, 0, 7, 2, 33, 5] * 7]
            pieces[4] = pieces[4][::2]  # a strided piece
            got = engine.cat_rows(pieces)
            assert torch.equal(got, torch.cat(pieces, 0)), (dt, trail)


def test_concurrent_partition_runs_match_sequential():
    """engine.run_programs_concurrent issues the partitions of one program on
    up to 4 side streams: results must equal a plain sequential run, over
    repeated iterations where the zero-copy captures are replayed from a
    different stream each time (partition i lands on stream (i + it) % 4)."""
    rng = np.random.default_rng(7)
    c = rng.standard_normal((16, 32))
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, [None, 32], name="x")
        d = tf.reduce_sum(tf.square(x), [1], keep_dims=True) - 2 * tf.matmul(x, tf.constant(c), transpose_b=True)
        idx = tf.argmin(d, 1, name="i")
        tf.unsorted_segment_sum(x, idx, 16, name="s")
        tf.reduce_sum(tf.unsorted_segment_sum(tf.ones_like(d), idx, 16), [1], name="n")
        tf.reduce_min(d, [1], name="m")
    prog = engine.program(g.serialize(), ["i", "s", "n", "m"], ["x"])
    dev = torch.device("cuda", 0)
    parts = [torch.randn((20000 + 1000 * k, 32), dtype=torch.float64, device=dev) for k in range(5)]
    for it in range(6):
        order = parts[it % 5:] + parts[:it % 5]  # rotate: each partition changes stream
        got = engine.run_programs_concurrent(prog, [[p] for p in order], dev)
        for p, outs in zip(order, got):
            xin = p.cpu().numpy()
            dd = (xin ** 2).sum(1, keepdims=True) - 2 * xin @ c.T
            want_i = dd.argmin(1)
            np.testing.assert_array_equal(outs[0].cpu().numpy(), want_i)
            want_s = np.zeros((16, 32))
            np.add.at(want_s, want_i, xin)
            np.testing.assert_allclose(outs[1].cpu().numpy(), want_s, rtol=1e-9, atol=1e-8)
            np.testing.assert_allclose(outs[3].cpu().numpy(), dd.min(1), rtol=1e-9, atol=1e-9)
        for p in parts:
            p.mul_(0.99)


def test_map_blocks_concurrent_partitions_frame():
    """A device-cached frame of 4 partitions: map_blocks runs them side by side
    and the frame result equals the CPU result."""
    xs = np.random.default_rng(8).standard_normal((40000, 8))
    df = tfs.from_columns({"x": xs}, num_partitions=4).cache_on_device()
    before = engine.metrics.snapshot().get("concurrent_partition_runs", 0)
    tfs.set_config(concurrent_partitions=True)
    try:
        with tf.Graph().as_default():
            xb = tf.placeholder(tf.float64, [None, 8], name="x")
            z = tf.reduce_sum(xb * xb, [1], name="z")
            out = tfs.map_blocks(z, df)
            got = out.to_numpy("z")
    finally:
        tfs.set_config(concurrent_partitions=False)
    assert engine.metrics.snapshot().get("concurrent_partition_runs", 0) - before == 4
    np.testing.assert_allclose(got, (xs * xs).sum(1), rtol=1e-12)


def test_zero_copy_replay_outputs_alias_graph_buffers_when_released():
    """The iterative pattern (outputs dropped before the next run): one
    instance per address, replayed every time with no output copy, and the
    results stay right while inputs change in place."""
    rng = np.random.default_rng(9)
    c = rng.standard_normal((10, 64))
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, [None, 64], name="x")
        d = tf.reduce_sum(tf.square(x), [1], keep_dims=True) - 2 * tf.matmul(x, tf.constant(c), transpose_b=True)
        idx = tf.argmin(d, 1, name="i")
        tf.unsorted_segment_sum(x, idx, 10, name="s")
        tf.reduce_min(d, [1], name="m")
    prog = engine.program(g.serialize(), ["i", "s", "m"], ["x"])
    dev = torch.device("cuda", 0)
    p = torch.randn((30000, 64), dtype=torch.float64, device=dev)
    before = prog.stats()
    for it in range(10):
        p.mul_(1.02)
        i, sm, m = engine.run_program(prog, [p], dev)
        xin = p.cpu().numpy()
        dd = (xin ** 2).sum(1, keepdims=True) - 2 * xin @ c.T
        np.testing.assert_array_equal(i.cpu().numpy(), dd.argmin(1))
        np.testing.assert_allclose(m.cpu().numpy(), dd.min(1), rtol=1e-9, atol=1e-9)
        del i, sm, m
    st = prog.stats()
    assert st["graphs_captured"] - before["graphs_captured"] == 1
    assert st["graph_replays"] - before["graph_replays"] >= 7
    assert st["graph_busy"] - before["graph_busy"] == 0


def test_cat_rows_many_matches_torch_cat():
    """Several columns concatenated in one launch: each result equals
    torch.cat of its pieces (mixed dtypes, trailing shapes, a strided piece)."""
    dev = torch.device("cuda", 0)
    a = [torch.randn((n, 3, 5), dtype=torch.float64, device=dev) for n in (7, 1, 30, 2)]
    b = [torch.randint(-9, 9, (n,), dtype=torch.int32, device=dev) for n in (7, 1, 30, 2)]
    c = [torch.randn((5, n), device=dev).t() for n in (7, 1, 30, 2)]  # non-contiguous pieces
    got = engine.cat_rows_many([a, b, c])
    for g, parts in zip(got, (a, b, c)):
        want = torch.cat(parts, 0)
        assert g.shape == want.shape and g.dtype == want.dtype
        torch.testing.assert_close(g, want, rtol=0, atol=0)


def test_zero_copy_replay_waits_for_a_recorded_side_stream_reader():
    """An aliased replay output read on a side stream (engine.record_stream)
    and dropped on the host before that read ran: the next replay must wait
    for the side stream instead of rewriting the buffer under the reader
    (executor.cpp PtrCap::wait_uses)."""
    from tensorframes_amd._native import _C
    rng = np.random.default_rng(11)
    c = rng.standard_normal((10, 64))
    g = tf.Graph()
    with g.as_default():
        x = tf.placeholder(tf.double, [None, 64], name="x")
        d = tf.reduce_sum(tf.square(x), [1], keep_dims=True) - 2 * tf.matmul(x, tf.constant(c), transpose_b=True)
        idx = tf.argmin(d, 1, name="i")
        tf.unsorted_segment_sum(x, idx, 10, name="s")
        tf.reduce_min(d, [1], name="m")
    prog = engine.program(g.serialize(), ["i", "s", "m"], ["x"])
    dev = torch.device("cuda", 0)
    p = torch.randn((30000, 64), dtype=torch.float64, device=dev)
    for _ in range(4):  # warm, capture, first aliased replays
        outs = engine.run_program(prog, [p], dev)
        del outs
    before = prog.stats()
    i, sm, m = engine.run_program(prog, [p], dev)
    assert prog.stats()["graph_replays"] - before["graph_replays"] == 1  # an aliased replay
    want = m.cpu().clone()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        _C.device_stall(0.4)  # the reader is delayed
        seen = torch.empty_like(m)
        seen.copy_(m)
    engine.record_stream(m, side)
    del i, sm, m
    p.mul_(3.0)  # new inputs: the next replay writes different values
    i2, sm2, m2 = engine.run_program(prog, [p], dev)
    torch.cuda.synchronize()
    assert prog.stats()["graph_busy"] - before["graph_busy"] == 0  # the buffers were reused (aliased)
    assert torch.equal(seen.cpu(), want)  # the reader saw the old values
    assert not torch.equal(m2.cpu(), want)

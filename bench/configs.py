"""Benchmarks for every BASELINE.json config (the headline config 3 is
/bench.py at the repo root).

    python bench/configs.py plumbing            # 1: 10-row double DF, map_blocks Add(+3), CPU
    python bench/configs.py add                 # 2: 1M x float32[128] map_blocks Add, 1 GPU
    python bench/configs.py reduce              # 4: 10M x float32[1024] reduce_blocks Sum
    python bench/configs.py inception           # 5: N x 224x224x3 Inception-v3 scoring
    python bench/configs.py kmeans              # reference demo workload
    python bench/configs.py reduce --gpus N     # N ranks, one per GPU (spawned here)
    torchrun --nproc-per-node N bench/configs.py reduce|inception ...

Each prints one JSON line (rank 0). Data is synthetic, weights random-init.
With `--gpus N > 1` outside torchrun the parent process starts N fresh ranks
(tensorframes_amd/parallel/launch.py) and never touches the GPU itself.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# the package (and its HIP runtime) is imported by the ranks only: see main()
tfs = tf = engine = _C = Block = dist = None
ArrayType = FloatType = StructField = StructType = None


def _import_package():
    global tfs, tf, engine, _C, Block, dist, ArrayType, FloatType, StructField, StructType
    import tensorframes_amd as _tfs
    from tensorframes_amd import engine as _engine, tf as _tf
    from tensorframes_amd._native import _C as __C
    from tensorframes_amd.frame.block import Block as _Block
    from tensorframes_amd.frame import types as _types
    from tensorframes_amd.parallel import dist as _dist
    tfs, tf, engine, _C, Block, dist = _tfs, _tf, _engine, __C, _Block, _dist
    ArrayType, FloatType, StructField, StructType = (_types.ArrayType, _types.FloatType, _types.StructField,
                                                     _types.StructType)


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    dist.barrier()


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    sync()
    _C.roctx_push("tfa.timed_steps")  # rocprofv3 --marker-trace: the timed window
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    dt = time.perf_counter() - t0
    _C.roctx_pop()
    if dist.is_distributed():
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce_(t, "Max")
        dt = float(t.item())
    return dt / steps


_ARGS = {}


def emit(d):
    """One JSON line on rank 0, in bench.py's schema (n_gpus, steps, warmup,
    ms_per_step, higher_is_better) so the driver can check it the same way."""
    if dist.rank() == 0:
        d.setdefault("n_gpus", dist.world_size() if torch.cuda.is_available() else 0)
        d.setdefault("steps", _ARGS.get("steps"))
        d.setdefault("warmup", _ARGS.get("warmup"))
        d.setdefault("higher_is_better", True)
        from tensorframes_amd.utils.sysinfo import box_id
        d.setdefault("box", box_id())
        print(json.dumps(d))


def vec_schema(name="x", dim=None):
    return StructType([tfs.tensor_field(name, tf.float32, [dim])])


def gen_frame(rows, dim, nparts, pinned, device=None, name="x"):
    """Synthetic float32[dim] frame: pinned host memory or device-resident."""
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None

    def make(p):
        a, b = (p * rows) // nparts, ((p + 1) * rows) // nparts
        if device is not None:
            t = torch.randn((b - a, dim), device=device, generator=torch.Generator(device=device).manual_seed(p))
            return Block(b - a, {name: t})
        host = _C.empty_pinned([b - a, dim], torch.float32) if pinned else torch.empty((b - a, dim))
        step = 1 << 20
        for s in range(0, b - a, step):
            e = min(b - a, s + step)
            src = torch.randn((e - s, dim), device=dev) if dev is not None else torch.randn((e - s, dim))
            host[s:e].copy_(src)
        return Block(b - a, {name: host})
    return tfs.generate(vec_schema(name, dim), nparts, make).cache()


# ------------------------------------------------------------------ configs
def cfg_plumbing(a):
    tfs.set_config(device="cpu")
    df = tfs.create_dataframe([tfs.Row(x=float(i)) for i in range(10)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")

        def step():
            assert tfs.map_blocks(z, df).collect()[0].z == 3.0
        ms = timed(step, a.steps, a.warmup) * 1e3
    emit({"config": "1: 10-row double DF, map_blocks Add(+3), CPU plumbing", "metric": "latency",
          "value": ms, "unit": "ms/call", "higher_is_better": False, "device": "cpu"})


def cfg_refperf(a):
    """The reference's perf suites (all `ignore`d there, timings printed, never
    recorded; src/test/scala/org/tensorframes/perf/*.scala):
      PerformanceSuite:14-26        20M-row range DF, map_blocks x+x, then a sum, x10
      ConvertPerformanceSuite:19-63 rows -> tensor, 10M Int scalar cells / one 10M vector
      ConvertBackPerformanceSuite   tensor -> rows, 10M Int cells
    Here the conversions are Arrow columns <-> block tensors (the engine's
    columnar path) and Python Row objects -> frame (the boxed path)."""
    import pyarrow as pa
    n = a.rows or 20_000_000
    nparts = max(1, dist.world_size()) * 4
    df = tfs.range(n, num_partitions=nparts).cache()
    df.local_blocks()
    with tf.Graph().as_default():
        x = tfs.block(df, "id", tf_name="id")
        y = tf.add(x, x, name="y")
    with tf.Graph().as_default():
        yi = tf.placeholder(tf.int64, [None], name="y_input")
        total = tf.reduce_sum(yi, [0], name="y")

    def step():
        out = tfs.map_blocks(y, df, trim=True)
        s = tfs.reduce_blocks(total, out)
        assert int(s) == n * (n - 1)
    t_map = timed(step, a.steps, a.warmup)
    # rows -> tensor: 10M int32 cells from an Arrow column (zero-copy block tensors)
    cells = 10_000_000
    col = pa.array(np.arange(cells, dtype=np.int32))
    t_conv = timed(lambda: tfs.from_arrow(pa.table({"x": col}), 1).local_blocks(), a.steps, a.warmup)
    vec = pa.FixedSizeListArray.from_arrays(col, cells)  # one 10M-element vector cell
    t_conv_vec = timed(lambda: tfs.from_arrow(pa.table({"x": vec}), 1).local_blocks(), a.steps, a.warmup)
    # tensor -> rows: 10M int32 cells back to an Arrow column
    back = tfs.from_columns({"x": np.arange(cells, dtype=np.int32)}, num_partitions=1).cache()
    back.local_blocks()
    t_back = timed(lambda: back.to_arrow(), a.steps, a.warmup)
    # tensor -> Row objects (the reference's ConvertBackPerformanceSuite:22-43 case,
    # a real Row per cell: native build_rows, runtime/packer.cpp)
    t_back_rows = timed(lambda: back.collect(), 3, 1)
    # boxed path (the reference's ConvertPerformanceSuite:19-39 case): 10M Row(int)
    # objects -> an int column, through the native packer (runtime/packer.cpp)
    rows = [tfs.Row(x=i) for i in range(10_000_000)]
    t_rows = timed(lambda: tfs.create_dataframe(rows, num_partitions=1).local_blocks(), 3, 1)
    emit({"config": "reference perf suites (PerformanceSuite / Convert / ConvertBack)",
          "map_blocks_x_plus_x_then_sum_20M_rows_ms": t_map * 1e3,
          "map_blocks_x_plus_x_then_sum_rows_per_sec": n / t_map,
          "convert_10M_int_cells_arrow_zero_copy_view_ms": t_conv * 1e3,
          "convert_one_10M_vector_arrow_zero_copy_view_ms": t_conv_vec * 1e3,
          "convert_back_10M_int_cells_to_arrow_ms": t_back * 1e3,
          "convert_back_10M_int_cells_to_python_Rows_ms": t_back_rows * 1e3,
          "convert_back_10M_int_cells_to_python_Rows_rows_per_sec": cells / t_back_rows,
          "convert_10M_python_Row_int_cells_ms": t_rows * 1e3,
          "convert_10M_python_Row_int_cells_rows_per_sec": 10_000_000 / t_rows,
          "device": str(engine.compute_device()), "data": "synthetic"})


def cfg_add(a):
    rows, dim = a.rows or 1_000_000, 128
    nparts = max(1, dist.world_size()) * 4
    res = {}
    for mode in ("host", "device"):
        df = gen_frame(rows, dim, nparts, pinned=True,
                       device=torch.device("cuda", torch.cuda.current_device()) if mode == "device" else None)
        df.local_blocks()
        with tf.Graph().as_default():
            x = tfs.block(tfs.analyze(df) if False else df, "x")
            y = tf.add(x, 1.0, name="y")

            def step():
                tfs.map_blocks(y, df, trim=True).local_blocks()
            res[mode] = timed(step, a.steps, a.warmup)
    emit({"config": "2: 1M-row float32[128] map_blocks Add, 1 MI355X", "metric": "rows/sec",
          "value": rows / res["host"], "unit": "rows/s", "higher_is_better": True,
          "ms_per_step": res["host"] * 1e3, "device_resident_rows_per_sec": rows / res["device"],
          "device_resident_ms_per_step": res["device"] * 1e3,
          "device_resident_hbm_GBps": 2 * rows * dim * 4 / res["device"] / 1e9,
          "rows": rows, "dtype": "fp32", "data": "synthetic"})


def cfg_reduce(a):
    rows, dim = a.rows or 10_000_000, 1024
    nparts = max(1, dist.world_size()) * a.parts_per_gpu
    res = {}
    for mode in ("host", "device"):
        dev = torch.device("cuda", torch.cuda.current_device())
        df = gen_frame(rows, dim, nparts, pinned=True, device=dev if mode == "device" else None)
        df.local_blocks()
        with tf.Graph().as_default():
            xi = tf.placeholder(tf.float32, [None, dim], name="x_input")
            s = tf.reduce_sum(xi, [0], name="x")
            out = {}

            def step():
                out["v"] = tfs.reduce_blocks(s, df)
            res[mode] = timed(step, a.steps, a.warmup)
        del df
        torch.cuda.empty_cache()
    comb = ("RCCL all-reduce" if dist.is_distributed() and dist.gpu_collectives() else
            "gloo all-reduce" if dist.is_distributed() else "none (1 rank, no collective)")
    emit({"config": f"4: {rows}-row float32[1024] reduce_blocks ReduceSum, {nparts} partitions on "
                    f"{dist.world_size()} GPU rank(s); cross-rank combine: {comb}",
          "collective_device_ms_total": dist.collective_device_ms() if dist.is_distributed() else 0.0,
          "metric": "rows/sec", "value": rows / res["host"], "unit": "rows/s", "higher_is_better": True,
          "ms_per_step": res["host"] * 1e3, "device_resident_rows_per_sec": rows / res["device"],
          "device_resident_ms_per_step": res["device"] * 1e3, "rows": rows,
          "parallelism": f"dp{dist.world_size()}", "dtype": "fp32", "data": "synthetic"})


def cfg_inception(a):
    """Config 5: map_blocks Inception-v3 scoring of an image column.

    --source host (default for the BASELINE scale): a 1M-row 224x224x3 column
    in page-locked HOST memory, streamed partition by partition (lazily
    generated, never materialised whole: 1M f32 images are 602 GB) through
    the pipelined H2D / compute / D2H chunk loop; the probabilities
    [rows, 1000] come back to host memory. Partitions cycle through a ring of
    `--ring` distinct synthetic pinned partitions (generated once, untimed),
    so the timed region has no generation work.
    --input-dtype uint8: the column holds decoded uint8 pixels (the reference
    decodes JPEGs to uint8: src/main/python/tensorframes_snippets/read_image.py:42);
    the graph casts and normalises them on the device (one fused kernel),
    a quarter of the PCIe bytes.
    --source device: images generated directly in HBM (kernel rate, no PCIe)."""
    from tensorframes_amd.models import cnn
    size = a.image_size
    world = max(1, dist.world_size())
    host = a.source == "host"
    images = a.rows or (1_000_000 if host else 16384 * world)
    batch = a.batch or (2048 if host else 4096)
    nparts = max(1, -(-images // batch))
    u8 = a.input_dtype == "uint8"
    dev = torch.device("cuda", torch.cuda.current_device())
    tdt = torch.uint8 if u8 else torch.float32
    with tf.Graph().as_default() as g:
        if u8:
            img = tf.placeholder(tf.uint8, [None, size, size, 3], name="image")
            x = (tf.cast(img, tf.float32) * (2.0 / 255.0)) - 1.0  # fused: one kernel
            g, iname, oname = cnn.inception_v3(image_size=size, inputs=x)
        else:
            g, iname, oname = cnn.inception_v3(image_size=size, graph=g)
    schema = StructType([tfs.tensor_field("image", tf.uint8 if u8 else tf.float32, [size, size, 3])])

    def rows_of(p):
        return ((p + 1) * images) // nparts - (p * images) // nparts

    def synth(n, seed):
        gen = torch.Generator(device=dev).manual_seed(seed)
        if u8:
            return torch.randint(0, 256, (n, size, size, 3), device=dev, dtype=torch.uint8, generator=gen)
        return torch.rand((n, size, size, 3), device=dev, generator=gen)

    if host:
        tfs.set_config(chunk_bytes=a.chunk_images * size * size * 3 * (1 if u8 else 4), min_pipeline_chunks=1)
        ring = []
        for k in range(min(a.ring, nparts)):
            buf = _C.empty_pinned([max(rows_of(p) for p in range(min(nparts, a.ring + 1))), size, size, 3], tdt)
            for s0 in range(0, buf.shape[0], 256):
                e0 = min(buf.shape[0], s0 + 256)
                buf[s0:e0].copy_(synth(e0 - s0, 1000 * k + s0))
            ring.append(buf)
        torch.cuda.synchronize()

        def make(p):
            return Block(rows_of(p), {"image": ring[p % len(ring)][:rows_of(p)]})
    else:
        def make(p):
            return Block(rows_of(p), {"image": synth(rows_of(p), p)})
    df = tfs.generate(schema, nparts, make)
    warm = tfs.generate(schema, min(nparts, 2 * world), make)
    prob = g.get_tensor_by_name(oname + ":0")

    def run(frame):
        return tfs.map_blocks(prob, frame, trim=True).count()
    for _ in range(max(1, a.warmup)):
        run(warm)  # plans, GEMM tile tuning, fused-kernel JIT
    from tensorframes_amd.utils.logging import metrics
    metrics.reset()
    dt = timed(lambda: run(df), a.steps, 0)
    m = metrics.snapshot()
    if a.step_profile:  # one more, untimed step with per-step device timing
        from tensorframes_amd.utils.profiling import step_profile
        step_profile(lambda: run(df), a.step_profile,
                     f"Inception-v3, {images} images ({a.source}-resident, batch {batch}): per-layer device time")
    flops_per_image = _inception_flops(size)
    in_bytes = images * size * size * 3 * (1 if u8 else 4)
    emit({"config": f"5: {images}-row {size}x{size}x3 {a.input_dtype} image column ({a.source}-resident), "
                    f"map_blocks Inception-v3 scoring on {world} GPU rank(s)",
          "metric": "images/sec", "value": images / dt, "unit": "images/s", "higher_is_better": True,
          "ms_per_step": dt * 1e3, "rows": images, "partitions": nparts, "partition_rows": batch,
          "chunk_images": a.chunk_images if host else None, "tflops": images * flops_per_image / dt / 1e12,
          "input_GBps": in_bytes / dt / 1e9 if host else None, "pipelined_chunks": m.get("chunks"),
          "parallelism": f"dp{world}", "dtype": "fp32", "input_dtype": a.input_dtype,
          "compute_precision": a.precision,
          "data": ("synthetic images in page-locked host memory (ring of %d partitions); " % a.ring if host else
                   "synthetic images generated in HBM; ") + "random-init frozen Inception-v3"})


def _inception_flops(size):
    """2*MACs of the conv/matmul layers, from the graph's own shapes."""
    from tensorframes_amd.models import cnn
    g, _, _ = cnn.inception_v3(image_size=size)
    total = 0
    for op in g.get_operations():
        if op.type == "Conv2D":
            out = op.outputs[0].get_shape().as_list()
            w = op.inputs[1].get_shape().as_list()
            total += 2 * out[1] * out[2] * out[3] * w[0] * w[1] * w[2]
        elif op.type == "MatMul":
            w = op.inputs[1].get_shape().as_list()
            total += 2 * w[0] * w[1]
    return total


def cfg_kmeans(a):
    from tensorframes_amd.models import kmeans
    n, f, k = a.rows or 100_000, 100, 10
    rng = np.random.default_rng(2)
    pts = rng.uniform(0.0, 1.0, size=(n, f))
    df = tfs.analyze(tfs.from_columns({"features": pts}, num_partitions=max(1, dist.world_size()) * 4)).cache()
    c0 = np.random.default_rng(2).standard_normal((k, f))
    frames = {"host": df}
    if engine.gpu_available():
        # iterative workloads keep the staged partitions in HBM
        frames["device"] = df.cache_on_device(engine.compute_device())
    out = {}
    for where, frame in frames.items():
        for variant, agg in (("aggregate", False), ("in_graph", True)):
            kmeans.kmeans(frame, c0, num_iters=max(a.warmup, 1), tf_aggregate=agg)  # plans, tile tuning
            t0 = time.perf_counter()
            c, ds = kmeans.kmeans(frame, c0, num_iters=a.steps, tf_aggregate=agg)
            out[f"{variant}_{where}"] = (time.perf_counter() - t0) / max(len(ds), 1) * 1e3
    best = out.get("in_graph_device", out["in_graph_host"])
    emit({"config": "K-Means 100k x 100, k=10 (reference demo)", "metric": "ms/iteration",
          "value": best, "unit": "ms", "higher_is_better": False,
          **{f"{k}_ms": v for k, v in out.items()}})



def _launcher():
    """parallel/launch.py loaded by path: the launcher parent imports neither
    the package nor its HIP runtime (it never touches the GPU)."""
    import importlib.util
    root = os.path.dirname(os.path.abspath(__file__))
    if os.path.basename(root) == "bench":
        root = os.path.dirname(root)
    spec = importlib.util.spec_from_file_location(
        "_tfa_launch", os.path.join(root, "tensorframes_amd", "parallel", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["plumbing", "add", "reduce", "inception", "kmeans", "refperf"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--parts-per-gpu", type=int, default=1)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batch", type=int, default=None,
                    help="rows per partition (inception: default 4096 device-resident, 2048 host-resident; "
                         "device 25.46k / 25.20k / 24.80k img/s at 4096 / 2048 / 1024, profiles/r6_validate/sweep/)")
    ap.add_argument("--source", choices=["host", "device"], default="host", help="inception: where the column lives")
    ap.add_argument("--step-profile", default="", help="inception: after the timed steps, one more step with "
                    "per-step device timing, written to this JSON (+ .md)")
    ap.add_argument("--input-dtype", choices=["float32", "uint8"], default="float32", help="inception image dtype")
    ap.add_argument("--chunk-images", type=int, default=2048,
                    help="inception (host): images per pipelined chunk (1M rows: 25.28k vs 24.94k img/s at 1024, "
                         "profiles/r6_validate/sweep/)")
    ap.add_argument("--ring", type=int, default=3, help="inception (host): distinct synthetic partitions")
    ap.add_argument("--precision", choices=["f32", "bf16x3", "bf16"], default="f32",
                    help="float32 MatMul/Conv2D compute mode (Config.precision); f32 = exact")
    ap.add_argument("--gpus", type=int, default=1, help="ranks to spawn (one per GPU) outside torchrun")
    ap.add_argument("--force-collectives", action="store_true",
                    help="run the cross-rank collectives even with one rank (RCCL group of size 1)")
    a = ap.parse_args()
    _ARGS.update(steps=a.steps, warmup=a.warmup)
    spawn_if_needed = _launcher().spawn_if_needed
    rc = spawn_if_needed(a.gpus)
    if rc is not None:
        sys.exit(rc)
    _import_package()
    from tensorframes_amd.utils import faults
    faults.exit_on_device_fault(_rank_main)(a)


def _rank_main(a):
    tfs.set_config(precision=a.precision)
    dist.init(force=a.force_collectives)
    if torch.cuda.is_available():
        torch.cuda.set_device(dist.local_rank() % torch.cuda.device_count())
        dist.bind_numa()
    {"plumbing": cfg_plumbing, "add": cfg_add, "reduce": cfg_reduce, "inception": cfg_inception,
     "kmeans": cfg_kmeans, "refperf": cfg_refperf}[a.config](a)
    dist.shutdown()


if __name__ == "__main__":
    main()

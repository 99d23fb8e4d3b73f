"""Headline benchmark: rows/sec of `map_blocks` MatMul(512x512)+Relu over a
10M-row float32[512] DataFrame (BASELINE.json config 3, the north-star metric
"rows/sec map_blocks MatMul on 10M-row DF at 1/2/4/8 MI355X").

    python bench.py --gpus N --steps K --warmup W          (spawns N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

With `--gpus N > 1` and no torchrun environment, the parent process never
touches the GPU: it starts N fresh child processes (parallel/launch.py), one
rank per GPU, and exits with their status.

The 10M rows are split over the ranks (strong scaling: total work fixed),
4 partitions per rank. Data is synthetic (random normal) and the weights are
random-init; both are generated outside the timed region.

One step = one full `map_blocks` pass, materialised: every partition's
float32[512] input is read from the DataFrame's page-locked host memory,
staged to HBM, multiplied by W (one fused MFMA GEMM+ReLU kernel per chunk)
and the float32[512] output column is written back to page-locked host
memory (PCIe traffic both ways is inside the timed region).

`--mode device` additionally times the same pass on a DataFrame cached in
HBM (`cache_on_device()`, outputs stay in HBM) and reports it as an extra
field; the headline `value` is always the host-resident pass.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as torch_dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_VALUE = None  # the reference publishes no number
TOTAL_ROWS = 10_000_000
DIM = 512


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=TOTAL_ROWS)
    ap.add_argument("--parts-per-gpu", type=int, default=4)
    ap.add_argument("--mode", choices=["host", "device", "both"], default="both")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: rehearse the launcher/collectives on the host (gloo), e.g. in CPU tests")
    return ap.parse_args()



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

def _chosen_tiles():
    """The f32 tiles the MatMul ran on: per GEMM shape (M, N, K) the tile in
    force (kernels/gemm.hip autotuner, started from the shipped gfx950
    defaults in tensorframes_amd/tiles/gfx950.json)."""
    from tensorframes_amd import _native
    _C = _native._C
    out = []
    for key, tile in _C.gemm_tune_table():
        if key[1] == DIM and key[2] == DIM:
            bm, bn, core = _C.gemm_tile_dims(tile)
            dflt = [e["tile"] for e in _native.default_entries() if e["key"] == list(key)]
            out.append({"M": key[0], "N": key[1], "K": key[2], "tile": tile, "dims": f"{bm}x{bn}",
                        "core": "g2" if core == 2 else "round4", "default": dflt[0] if dflt else None})
    return out


def main():
    args = parse()
    spawn_if_needed = _launcher().spawn_if_needed
    extra = {"TFA_DEVICE": "cpu"} if args.device == "cpu" else None
    rc = spawn_if_needed(args.gpus, extra_env=extra)
    if rc is not None:  # we were the launcher parent; the ranks did the work
        sys.exit(rc)
    if args.device == "cpu":
        os.environ["TFA_DEVICE"] = "cpu"
    from tensorframes_amd.utils import faults
    # a rank that loses its GPU context exits with EXIT_DEVICE_FAULT, so the
    # launcher can re-run the job in fresh processes (TFA_MAX_RESTARTS)
    faults.exit_on_device_fault(rank_main)(args)


def rank_main(args):
    import tensorframes_amd as tfs
    from tensorframes_amd import tf
    from tensorframes_amd.frame.block import Block
    from tensorframes_amd.frame.types import ArrayType, FloatType, StructField, StructType
    from tensorframes_amd.parallel import dist
    from tensorframes_amd.utils.sysinfo import box_id

    use_gpu = args.device == "cuda"
    dist.init(backend=None if use_gpu else "gloo")
    rank, world = dist.rank(), dist.world_size()
    backend = dist.backend_name()
    # the multi-GPU numbers are only meaningful on the job the driver asked
    # for: N ranks over RCCL. A silent fallback (gloo, or fewer ranks) fails here.
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the job has {world} rank(s)")
    # TFA_BENCH_REHEARSAL=1 (with TFA_DIST_BACKEND=gloo): N ranks sharing one
    # GPU, where RCCL refuses duplicate devices; the JSON line says so
    rehearsal = os.environ.get("TFA_BENCH_REHEARSAL") == "1"
    if use_gpu and world > 1 and backend != "nccl" and not rehearsal:
        raise SystemExit(f"bench.py: GPU job with backend {backend!r}; expected 'nccl' (RCCL over xGMI)")
    if use_gpu:
        assert torch.cuda.is_available(), "bench.py needs a GPU (or --device cpu)"
        dev = torch.device("cuda", dist.local_rank() % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        numa_cpus = dist.bind_numa(dev.index)  # before any pinned allocation
    else:
        dev, numa_cpus = torch.device("cpu"), []

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    nparts = world * args.parts_per_gpu
    schema = StructType([tfs.tensor_field("x", tf.float32, [DIM])])

    # ---- synthetic data, generated on the GPU and staged into pinned host memory (untimed)
    from tensorframes_amd._native import _C

    def make(p):
        a, b = (p * args.rows) // nparts, ((p + 1) * args.rows) // nparts
        host = _C.empty_pinned([b - a, DIM], torch.float32) if use_gpu else torch.empty((b - a, DIM))
        gen = torch.Generator(device=dev).manual_seed(1000 + p)
        step = 1 << 20
        for s in range(0, b - a, step):
            e = min(b - a, s + step)
            host[s:e].copy_(torch.randn((e - s, DIM), device=dev, generator=gen))
        return Block(b - a, {"x": host})

    base = tfs.generate(schema, nparts, make).cache()
    blocks = base.local_blocks()  # materialise the synthetic frame once (untimed)

    g = torch.Generator().manual_seed(7)
    w = (torch.randn((DIM, DIM), generator=g) / np.sqrt(DIM)).numpy().astype(np.float32)
    with tf.Graph().as_default():
        x = tfs.block(base, "x")
        y = tf.nn.relu(tf.matmul(x, tf.constant(w)), name="y")

    def step_host():
        out = tfs.map_blocks(y, base, trim=True)
        return out.local_blocks()

    def timed(fn, steps, warmup, marker="tfa.timed_steps"):
        from tensorframes_amd._native import _C
        for _ in range(warmup):
            fn()
        sync()
        dist.barrier()
        if use_gpu:
            _C.roctx_push(marker)  # rocprofv3 --marker-trace: the timed window (scripts/trace_window.py)
        t0 = time.perf_counter()
        res = None
        for _ in range(steps):
            res = None  # a step's output frame is dropped before the next step (like a loop body)
            res = fn()
        sync()
        dist.barrier()
        dt = time.perf_counter() - t0
        if use_gpu:
            _C.roctx_pop()
        own_dt = dt
        if dist.is_distributed():
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce_(t, "Max")
            dt = float(t.item())
        return dt, own_dt, res

    results, own = {}, {}
    dt, own["host"], res = timed(step_host, args.steps, args.warmup)
    # correctness spot check on a few rows of the first local partition
    pid = min(res)
    xin = blocks[pid].columns["x"][:64].double()
    ref = torch.clamp_min(xin @ torch.as_tensor(w).double(), 0)
    err = (res[pid].columns["y"][:64].double() - ref).abs().max().item()
    assert err < 1e-3, f"wrong result: max abs err {err}"
    results["host"] = dt

    dev_rows_per_s = None
    if args.mode in ("device", "both") and use_gpu:
        base_dev = base.cache_on_device(dev)

        def step_dev():
            return tfs.map_blocks(y, base_dev, trim=True).local_blocks()
        ddt, own["device"], _ = timed(step_dev, args.steps, args.warmup, "tfa.timed_steps_device")
        dev_rows_per_s = args.rows * args.steps / ddt
        results["device"] = ddt
        del base_dev

    ms = results["host"] / args.steps * 1e3
    value = args.rows * args.steps / results["host"]
    # one diagnostic line per rank on stderr (the driver's 8-GPU run is
    # diagnosable from its log): placement, backend, page-locked memory, own time
    pool = _C.pinned_pool_stats() if use_gpu else {}
    print(json.dumps({"bench_rank": rank, "local_rank": dist.local_rank(), "world_size": world,
                      "backend": backend, "device": str(dev),
                      "numa_cpus": (f"{min(numa_cpus)}-{max(numa_cpus)}" if numa_cpus else None),
                      "numa_cpu_count": len(numa_cpus),
                      "pinned_live_bytes": pool.get("live"), "pinned_peak_bytes": pool.get("peak"),
                      "pinned_cap_bytes": pool.get("limit"),
                      "own_ms_per_step": own["host"] / args.steps * 1e3,
                      "own_device_ms_per_step": (own["device"] / args.steps * 1e3) if "device" in own else None,
                      "rows": sum(b.nrows for b in blocks.values()), "partitions": sorted(blocks)}),
          file=sys.stderr, flush=True)
    if rank == 0:
        out = {
            "metric": "rows/sec map_blocks MatMul on 10M-row DF at 1/2/4/8 MI355X",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            "dtype": "fp32",
            "device": args.device,
            "data": "synthetic (random normal float32[512] rows in page-locked host memory; random-init W)",
            "config": {
                "model": "map_blocks relu(matmul(x[?,512], W[512,512])) float32",
                "global_batch": args.rows,
                "seq_len": DIM,
                "parallelism": f"dp{world}",
                "partitions": nparts,
                "rows": args.rows,
            },
            "device_resident_rows_per_sec": dev_rows_per_s,
            "device_resident_ms_per_step": None if dev_rows_per_s is None else results["device"] / args.steps * 1e3,
            "gemm_tflops_device_resident": None if dev_rows_per_s is None else dev_rows_per_s * 2 * DIM * DIM / 1e12,
            "max_abs_err": err,
            "rank0_numa_bound_cpus": len(numa_cpus),
            "gemm_tiles": _chosen_tiles() if use_gpu else None,
            "box": box_id(),
        }
        if rehearsal:
            out["rehearsal"] = f"{world} ranks sharing one GPU over {backend} (not a multi-GPU number)"
        print(json.dumps(out))
    dist.shutdown()


if __name__ == "__main__":
    main()

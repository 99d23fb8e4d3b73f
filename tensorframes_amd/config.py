"""Runtime configuration (one dataclass, `TFA_*` environment overrides).

The reference has no flag system (configuration is spread over Spark conf,
sbt properties and a hard-coded UDAF buffer size; reference:
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:573)."""
from __future__ import annotations

import dataclasses
import os


def _env(name, default, cast):
    v = os.environ.get(name)
    if v is None:
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "yes", "on")
    return cast(v)


@dataclasses.dataclass
class Config:
    # "auto" (GPU when present), "cpu", "cuda"
    device: str = dataclasses.field(default_factory=lambda: _env("TFA_DEVICE", "auto", str))
    # where DataFrame.collect() delivers rows across ranks: "all" (every rank,
    # the SPMD-safe default) or a rank number (the Spark driver's view; the
    # other ranks get [])
    collect_to: str = dataclasses.field(default_factory=lambda: _env("TFA_COLLECT_TO", "all", str))
    # value-preserving algebraic GraphDef rewrites before planning (graph/rewrite.py)
    graph_rewrites: bool = dataclasses.field(default_factory=lambda: _env("TFA_GRAPH_REWRITES", True, bool))
    # a program for a graph that differs from an earlier one only in the values
    # of its parameter constants takes over that program's plans (engine.program)
    plan_reuse: bool = dataclasses.field(default_factory=lambda: _env("TFA_PLAN_REUSE", True, bool))
    # target bytes of one input column per pipelined chunk (host->device->host)
    chunk_bytes: int = dataclasses.field(default_factory=lambda: _env("TFA_CHUNK_BYTES", 128 << 20, int))
    # a pipelined job is cut into at least this many chunks (when chunks stay >= 4 MB)
    min_pipeline_chunks: int = dataclasses.field(default_factory=lambda: _env("TFA_MIN_PIPELINE_CHUNKS", 16, int))
    # ring depth of the copy/compute pipeline
    pipeline_depth: int = dataclasses.field(default_factory=lambda: _env("TFA_PIPELINE_DEPTH", 3, int))
    # partitions smaller than this run in one shot (no chunking)
    min_chunked_rows: int = dataclasses.field(default_factory=lambda: _env("TFA_MIN_CHUNKED_ROWS", 65536, int))
    # ... or at least this many input bytes (a partition of 2048 images is 1.2 GB:
    # one-shot it would copy in, compute, copy out with nothing overlapped)
    min_chunked_bytes: int = dataclasses.field(default_factory=lambda: _env("TFA_MIN_CHUNKED_BYTES", 32 << 20, int))
    # streaming actions hand derived operators groups of partitions of up to
    # this many input bytes (one pipeline ramp per group; memory bound)
    stream_group_bytes: int = dataclasses.field(default_factory=lambda: _env("TFA_STREAM_GROUP_BYTES", 4 << 30, int))
    # allocate map_blocks outputs in page-locked host memory (DMA target)
    pinned_outputs: bool = dataclasses.field(default_factory=lambda: _env("TFA_PINNED_OUTPUTS", True, bool))
    pinned_min_bytes: int = dataclasses.field(default_factory=lambda: _env("TFA_PINNED_MIN_BYTES", 1 << 20, int))
    # map_rows: cells at least this large run on the GPU, smaller ones on the host executor
    map_rows_gpu_min_elems: int = dataclasses.field(default_factory=lambda: _env("TFA_MAP_ROWS_GPU_MIN", 16384, int))
    # map_rows: run same-shaped rows as one block through the lifted row graph
    map_rows_vectorize: bool = dataclasses.field(default_factory=lambda: _env("TFA_MAP_ROWS_VECTORIZE", True, bool))
    # map_rows batch-of-one cut: rows whose cut tensors are concatenated into one batched run
    # (JPEG -> VGG-16 on MI355X, f32 / bf16x3: 64 rows 3.6 / 4.9 k img/s, 256 rows 3.9 / 6.3 k,
    # profiles/r5_img/; the 14x14 layers only fill the CUs at a few hundred images)
    map_rows_batch_rows: int = dataclasses.field(default_factory=lambda: _env("TFA_MAP_ROWS_BATCH", 256, int))
    # map_rows image scoring: the per-row decode -> resize -> crop -> normalise
    # part of a chunk runs as ONE ragged-batch kernel (core._ImagePrep)
    map_rows_batched_prestage: bool = dataclasses.field(
        default_factory=lambda: _env("TFA_MAP_ROWS_BATCHED_PRESTAGE", True, bool))
    # ... with its JPEG cells decoded by the native libjpeg thread pool straight
    # into the chunk's pinned buffer (runtime/jpeg_decode.cpp), no GIL held
    native_jpeg_decode: bool = dataclasses.field(default_factory=lambda: _env("TFA_NATIVE_JPEG", True, bool))
    # groupBy string keys longer than 8 bytes: 2 words per row (word 0, 62-bit
    # hash) verified per group, instead of one word per 8 bytes of the
    # longest key + length (ops/groupby.string_key_hashed)
    string_key_hash: bool = dataclasses.field(default_factory=lambda: _env("TFA_STRING_KEY_HASH", True, bool))
    # threads of the native decode pool (0: min(16, CPUs available))
    decode_threads: int = dataclasses.field(default_factory=lambda: _env("TFA_DECODE_THREADS", 0, int))
    # re-runs of a partition task after a runtime (non-validation) failure; 0 = fail fast
    task_retries: int = dataclasses.field(default_factory=lambda: _env("TFA_TASK_RETRIES", 0, int))
    # timeout of one collective (RCCL, one-shot, shared memory, gloo): past it
    # the waiting rank raises CollectiveError (parallel/comm.py)
    collective_timeout_s: float = dataclasses.field(default_factory=lambda: _env("TFA_COLLECTIVE_TIMEOUT_S", 600.0, float))
    # an RCCL collective still incomplete past the timeout plus a grace period,
    # with no thread waiting on it, ends the process (status 76) after
    # ncclCommAbort, so the launcher tears the job down; False: the
    # communicator is only marked failed (the next collective raises)
    collective_timeout_exit: bool = dataclasses.field(default_factory=lambda: _env("TFA_COLLECTIVE_TIMEOUT_EXIT", True, bool))
    # host-tensor collectives of the ranks of one node through a shared-memory
    # segment (csrc/comm ShmComm) instead of gloo: the data path of CPU-only
    # jobs, the row-count / flag exchanges of GPU jobs
    shm_collectives: bool = dataclasses.field(default_factory=lambda: _env("TFA_SHM_COLLECTIVES", True, bool))
    # bytes per rank of the shared segment (payloads move in rounds of this size)
    shm_slot_bytes: int = dataclasses.field(default_factory=lambda: _env("TFA_SHM_SLOT_BYTES", 8 << 20, int))
    # CPU executor: programs with fewer input elements run on one intra-op thread
    cpu_parallel_min_elems: int = dataclasses.field(default_factory=lambda: _env("TFA_CPU_PARALLEL_MIN_ELEMS", 4_000_000, int))
    # float32 MatMul / Conv2D compute mode on the GPU: "f32" (exact, default),
    # "bf16" (bf16 operands) or "bf16x3" (hi/lo bf16 split, ~16-bit operands);
    # f32 accumulation and f32 tensors in every mode (kernels/gemm_bf16.hip)
    precision: str = dataclasses.field(default_factory=lambda: _env("TFA_PRECISION", "f32", str))
    # run the cross-rank collectives even in a 1-rank job (an RCCL/gloo group of
    # world size 1): exercises the collective path on a single GPU
    force_collectives: bool = dataclasses.field(default_factory=lambda: _env("TFA_FORCE_COLLECTIVES", False, bool))
    # device collectives: "engine" (the engine's own communicator,
    # parallel/comm.py: one-shot IPC all-reduce for <= 64 KB, an RCCL
    # communicator of its own for the rest) or "torch" (torch.distributed)
    collective_backend: str = dataclasses.field(default_factory=lambda: _env("TFA_COLLECTIVE_BACKEND", "engine", str))
    # the single-hop IPC all-reduce for small payloads (kernels/oneshot.hip)
    oneshot_allreduce: bool = dataclasses.field(default_factory=lambda: _env("TFA_ONESHOT_ALLREDUCE", True, bool))
    # map_blocks over a frame cached in HBM (cache_on_device) launches its
    # partitions at the call instead of at the first action, when the feed
    # columns total at most `eager_device_map_bytes`: the GPU runs them while
    # the host builds what comes next (iterative workloads)
    eager_device_map: bool = dataclasses.field(default_factory=lambda: _env("TFA_EAGER_DEVICE_MAP", True, bool))
    eager_device_map_bytes: int = dataclasses.field(
        default_factory=lambda: _env("TFA_EAGER_DEVICE_MAP_BYTES", 1 << 30, int))
    # small device-resident partitions of one map_blocks run side by side on
    # up to 4 streams (engine.run_programs_concurrent). Off by default: on the
    # K-Means demo (4 x 25k rows, host-bound) the stream switches and events
    # cost more host time than the overlap saves (0.92 -> 1.12 ms/iteration,
    # profiles/r4_validation/kmeans_concurrency.md)
    concurrent_partitions: bool = dataclasses.field(default_factory=lambda: _env("TFA_CONCURRENT_PARTITIONS", False, bool))
    # large device-resident partitions (each >= concurrent_large_bytes of
    # input: GPU-bound plans) of one map_blocks run two at a time on two
    # streams: one partition's kernels fill the CUs the other's kernel tails
    # leave idle (Inception-v3, 8 x 2048 images: 24.47 -> 25.19 k img/s on one box,
    # profiles/r6_final/incep_dev_2streams_run*.log vs incep_dev_serial_same_box.log). Peak memory: two plans' activations.
    concurrent_large_partitions: bool = dataclasses.field(
        default_factory=lambda: _env("TFA_CONCURRENT_LARGE", True, bool))
    concurrent_large_bytes: int = dataclasses.field(
        default_factory=lambda: _env("TFA_CONCURRENT_LARGE_BYTES", 64 << 20, int))
    concurrent_large_streams: int = dataclasses.field(
        default_factory=lambda: _env("TFA_CONCURRENT_LARGE_STREAMS", 2, int))
    # Winograd F(4,5) for the 5x5 stride-1 convs (Inception-v3 Mixed_5x b1_5x5:
    # 2.1x faster per layer, device-resident Inception 25.28 -> 25.88 k img/s,
    # profiles/r6_f45/). Opt-in: its f32 error (5.6e-7 of sum|a*b|) is 5.0x the
    # exact path's, above the 4x gate of the default-on Winograd kernels
    wino_5x5: bool = dataclasses.field(default_factory=lambda: _env("TFA_WINO_5X5", False, bool))
    # a 3x3 VALID MaxPool read only by a 1x1 conv runs inside the conv's kernel
    # (the pooled tensor never reaches HBM): Inception-v3's MaxPool_3a ->
    # Conv2d_3b 18.8 -> 13.9 ms per 8 x 2048 images, bitwise equal
    # (profiles/r6_poolconv/)
    pool_conv_fusion: bool = dataclasses.field(default_factory=lambda: _env("TFA_POOL_CONV_FUSION", True, bool))
    # synchronise + check after every kernel (debugging)
    debug_sync: bool = dataclasses.field(default_factory=lambda: _env("TFA_DEBUG_SYNC", False, bool))


config = Config()


def set_config(**kw):
    """Update `config` fields (`set_config(precision="bf16x3", task_retries=2)`);
    unknown keys raise AttributeError, a bad precision ValueError."""
    if "precision" in kw and kw["precision"] not in PRECISION_MODES:
        raise ValueError(f"precision must be one of {sorted(PRECISION_MODES)}, got {kw['precision']!r}")
    for k, v in kw.items():
        if not hasattr(config, k):
            raise AttributeError(f"unknown config key {k}")
        setattr(config, k, v)
    if "debug_sync" in kw:
        os.environ["TFA_DEBUG_SYNC"] = "1" if kw["debug_sync"] else "0"
        from ._native import _C
        _C.set_debug_sync(bool(kw["debug_sync"]))  # read by the executor on every launch
    if "precision" in kw:
        apply_precision()
    if "pool_conv_fusion" in kw:
        from ._native import _C
        from . import engine
        _C.set_pool_conv_fusion(bool(kw["pool_conv_fusion"]))
        engine.clear_program_cache()
    if "wino_5x5" in kw:
        from ._native import _C
        from . import engine
        _C.set_wino_5x5(bool(kw["wino_5x5"]))
        engine.clear_program_cache()  # plans hold (or lack) the F(4,5) filters


PRECISION_MODES = {"f32": 0, "bf16": 1, "bf16x3": 2}


def apply_precision():
    """Push `config.precision` to the native kernel library and drop cached
    plans (a captured HIP graph holds the kernels of the mode it was built in)."""
    if config.precision not in PRECISION_MODES:
        raise ValueError(f"precision must be one of {sorted(PRECISION_MODES)}, got {config.precision!r}")
    from ._native import _C
    from . import engine
    _C.set_f32_precision(PRECISION_MODES[config.precision])
    engine.clear_program_cache()

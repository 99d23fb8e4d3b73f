"""Per-layer device time of the plan that really runs (executor step timing,
csrc/runtime/executor.cpp set_step_timing): every step of every GPU plan run
inside `step_profile` gets a hipEvent pair; the records are summed per graph
node (over partitions / chunks) into a table of device ms, share of the step,
FLOPs and TFLOP/s, with the algorithm the step used (Winograd F(2x2,3x3) /
F(2,7), implicit GEMM, sibling-fused convs, fused elementwise regions).

    rows = step_profile(lambda: run(frame), "profiles/x/layers.json")

The timed numbers of a benchmark come from runs WITHOUT this (the events add
a few microseconds per step); a step-profile run is its own, extra step."""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, List, Optional

import torch

from .._native import _C


def step_profile(fn: Callable[[], object], path: Optional[str] = None, title: str = "") -> List[dict]:
    """Run fn() once with step timing on; returns the per-node rows (sorted by
    device ms) and, with `path`, writes them as JSON plus a markdown table
    next to it (same name, .md)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    _C.read_step_timing()  # drop stale records
    _C.set_step_timing(True)
    try:
        fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    finally:
        _C.set_step_timing(False)
    recs = _C.read_step_timing()
    rows = aggregate(recs)
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"title": title, "rows": rows, "steps_recorded": len(recs)}, f, indent=1)
        with open(os.path.splitext(path)[0] + ".md", "w") as f:
            f.write(markdown(rows, title))
    return rows


def aggregate(recs: List[dict]) -> List[dict]:
    by: Dict[tuple, dict] = {}
    order: List[tuple] = []
    for r in recs:
        key = (r["node"], r["op"], r["label"])
        e = by.get(key)
        if e is None:
            e = by[key] = {"node": r["node"], "op": r["op"], "algo": r["label"], "calls": 0, "ms": 0.0, "flops": 0.0,
                           "bytes": 0.0}
            order.append(key)
        e["calls"] += 1
        e["ms"] += float(r["ms"])
        e["flops"] += float(r["flops"])
        e["bytes"] += float(r.get("bytes", 0.0))
    total = sum(e["ms"] for e in by.values()) or 1.0
    rows = []
    for k in order:
        e = by[k]
        e["share"] = e["ms"] / total
        e["tflops"] = e["flops"] / (e["ms"] * 1e-3) / 1e12 if e["ms"] > 0 and e["flops"] else None
        # operands + outputs once each over the step's time: a step near the
        # HBM rate (~5-6 TB/s achievable) is memory-bound, whatever its TF/s
        e["min_GBps"] = e["bytes"] / (e["ms"] * 1e-3) / 1e9 if e["ms"] > 0 and e["bytes"] else None
        rows.append(e)
    rows.sort(key=lambda e: -e["ms"])
    return rows


def markdown(rows: List[dict], title: str = "") -> str:
    total = sum(e["ms"] for e in rows)
    flops = sum(e["flops"] for e in rows)
    out = [f"# {title}\n" if title else "",
           f"Sum of step device times: {total:.2f} ms; conv/GEMM FLOPs {flops / 1e12:.2f} T "
           f"({flops / (total * 1e-3) / 1e12 if total else 0:.1f} TFLOP/s over all steps).\n",
           "| node | op | algorithm | calls | ms | share | TFLOP/s | min GB/s |",
           "|---|---|---|---:|---:|---:|---:|---:|"]
    for e in rows:
        tf = f"{e['tflops']:.1f}" if e["tflops"] else ""
        bw = f"{e['min_GBps']:.0f}" if e.get("min_GBps") else ""
        out.append(f"| {e['node']} | {e['op']} | {e['algo']} | {e['calls']} | {e['ms']:.3f} | "
                   f"{100 * e['share']:.1f}% | {tf} | {bw} |")
    return "\n".join(out) + "\n"

"""Kernel breakdown of ONE timed window from a rocprofv3 run
(`--kernel-trace --marker-trace --output-format csv`): the window is the
roctx range bench/configs.py opens around its timed steps
("tfa.timed_steps"; warmup and autotuning stay outside it). Per kernel name:
dispatches, device ms, share of the window, mean us; plus how busy the GPU was
(union of kernel intervals / window).

    python scripts/trace_window.py gpurun_out/trace_incep --out profiles/r6_trace/incep_step.md
"""
import argparse
import csv
import glob
import json
import os
import re


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _col(row, *keys):
    for k in row:
        kl = k.lower()
        if any(kl == x for x in keys):
            return k
    for k in row:
        kl = k.lower()
        if any(x in kl for x in keys):
            return k
    raise KeyError(keys)


def window(marker_csv, marker):
    rows = _rows(marker_csv)
    for r in rows:
        if any(str(v).strip() == marker for v in r.values()):
            s, e = _col(r, "start_timestamp", "start"), _col(r, "end_timestamp", "end")
            return int(r[s]), int(r[e])
    raise SystemExit(f"no '{marker}' range in {marker_csv}")


def short(name):
    """the kernel name with its template arguments, without the parameter list"""
    name = name.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    name = re.sub(r"^void ", "", name)
    return name[:160]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="tfa.timed_steps")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    kcsv = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    mcsv = glob.glob(os.path.join(a.dir, "**", "*marker_api_trace.csv"), recursive=True)
    if not kcsv or not mcsv:
        raise SystemExit(f"kernel / marker trace CSVs not found under {a.dir}")
    t0, t1 = window(mcsv[0], a.marker)
    ks = _rows(kcsv[0])
    sk, ek, nk = _col(ks[0], "start_timestamp"), _col(ks[0], "end_timestamp"), _col(ks[0], "kernel_name")
    inside = [(int(r[sk]), int(r[ek]), r[nk]) for r in ks if int(r[sk]) >= t0 and int(r[ek]) <= t1]
    inside.sort()
    by = {}
    for s, e, n in inside:
        d = by.setdefault(short(n), {"kernel": short(n), "calls": 0, "ns": 0})
        d["calls"] += 1
        d["ns"] += e - s
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in inside:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    win = t1 - t0
    rows = sorted(by.values(), key=lambda d: -d["ns"])
    ktot = sum(d["ns"] for d in rows)
    summary = {"window_ms": win / 1e6, "kernels": len(inside), "kernel_ms": ktot / 1e6,
               "gpu_busy_pct": 100.0 * busy / win if win else 0.0}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(os.path.splitext(a.out)[0] + ".json", "w") as f:
        json.dump({"summary": summary, "kernels": [dict(d, ms=d["ns"] / 1e6) for d in rows]}, f, indent=1)
    lines = [f"# {a.title or 'one timed window'}\n",
             f"Window (roctx `{a.marker}`): {summary['window_ms']:.2f} ms; {summary['kernels']} kernel dispatches, "
             f"{summary['kernel_ms']:.2f} ms of kernel time; GPU busy {summary['gpu_busy_pct']:.1f}% of the window.\n",
             "| kernel | calls | ms | share of window | mean us |", "|---|---:|---:|---:|---:|"]
    for d in rows:
        lines.append(f"| `{d['kernel']}` | {d['calls']} | {d['ns'] / 1e6:.3f} | {100 * d['ns'] / win:.1f}% | "
                     f"{d['ns'] / d['calls'] / 1e3:.1f} |")
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(json.dumps(summary))


if __name__ == "__main__":
    main()

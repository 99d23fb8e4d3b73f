"""Summarise rocprofv3 --pmc passes of one GEMM/conv kernel (scripts/gpu_steps.sh
step `pmc`): per shape, the counters of the named kernel summed over its
dispatches, and the derived rates the round-4 verdict asks for:

  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                 (GRBM_GUI_ACTIVE is summed over the 8 XCDs: /8 = kernel cycles)
  mfma_cyc       SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA (64 for 32x32x2 f32)
  valu_per_mfma  (SQ_INSTS_VALU - SQ_INSTS_MFMA) / SQ_INSTS_MFMA (SQ_INSTS_VALU
                 counts the MFMAs too)
  lds_conflict   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_any / wait_inst / active   shares of SQ_WAVE_CYCLES

    python scripts/pmc_summary.py gpurun_out/pmc4 > profiles/r4_pmc/summary.md
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, match):
    agg = collections.defaultdict(float)
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            names.add(r["Kernel_Name"])
    return agg, names


def main():
    root = sys.argv[1]
    meta = json.load(open(os.path.join(root, "shapes.json")))
    out = []
    print("| shape | kernel | ms | TF/s | MFMA busy | cyc/MFMA | VALU/MFMA | LDS conflict | wait_any | wait_inst | active |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for s in meta:
        c = {}
        names = set()
        for p in ("a", "b"):
            agg, nm = load(os.path.join(root, f"{s['id']}{p}"), s["kernel"])
            for k, v in agg.items():
                c.setdefault(k, v)
            names |= nm
        t = {}
        tl = os.path.join(root, f"{s['id']}t.log")
        if os.path.exists(tl):
            for line in open(tl):
                if line.startswith("{"):
                    t = json.loads(line)
        g = lambda k: c.get(k, float("nan"))  # noqa: E731
        cyc = g("GRBM_GUI_ACTIVE") / 8
        row = dict(shape=s["name"], kernel=sorted(names)[0] if names else "?", ms=t.get("ms"), tflops=t.get("tflops"),
                   mfma_busy=g("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * cyc) if cyc else None,
                   mfma_cyc=g("SQ_VALU_MFMA_BUSY_CYCLES") / g("SQ_INSTS_MFMA"),
                   valu_per_mfma=(g("SQ_INSTS_VALU") - g("SQ_INSTS_MFMA")) / g("SQ_INSTS_MFMA"),
                   lds_conflict=g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"),
                   wait_any=g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
                   wait_inst=g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
                   active=g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES"),
                   counters=c)
        out.append(row)
        f = lambda v, fmt: (fmt % v) if isinstance(v, float) else str(v)  # noqa: E731
        print(f"| {row['shape']} | `{row['kernel'][:60]}` | {f(row['ms'], '%.3f')} | {f(row['tflops'], '%.1f')} | "
              f"{f(row['mfma_busy'], '%.3f')} | {f(row['mfma_cyc'], '%.1f')} | {f(row['valu_per_mfma'], '%.2f')} | "
              f"{f(row['lds_conflict'], '%.3f')} | {f(row['wait_any'], '%.3f')} | {f(row['wait_inst'], '%.3f')} | "
              f"{f(row['active'], '%.3f')} |")
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

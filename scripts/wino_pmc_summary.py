"""Summarise the `wino_pmc` step of scripts/gpu_steps.sh (three rocprofv3 --pmc
passes per layer of scripts/conv_layers.py: gpurun_out/wino_pmc/l<layer>_v<variant>_<pass>)
for the Winograd kernels: MFMA busy share, VALU / SALU / LDS instructions per
MFMA, LDS bank conflicts, wait shares, L2 hit rate.

    python scripts/wino_pmc_summary.py gpurun_out/wino_pmc > profiles/r6_wino/pmc_final.md
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d):
    agg = collections.defaultdict(float)
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "wino" not in r["Kernel_Name"]:
                continue
            names.add(re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")))
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return agg, names


def main():
    root = sys.argv[1]
    tags = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "l*_v*_*"))):
        tags[os.path.basename(d).rsplit("_", 2)[0]].append(d)
    print("| layer / variant | kernel | MFMA busy | VALU/MFMA | SALU/MFMA | LDS/MFMA | LDS conflict | wait_any | "
          "wait_inst | L2 hit |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for tag, dirs in sorted(tags.items()):
        c, names = {}, set()
        for d in dirs:
            agg, nm = load(d)
            for k, v in agg.items():
                c.setdefault(k, v)
            names |= nm
        g = lambda k: c.get(k, float("nan"))  # noqa: E731
        cyc = g("GRBM_GUI_ACTIVE") / 8
        mf = g("SQ_INSTS_MFMA")
        row = [g("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * cyc), (g("SQ_INSTS_VALU") - mf) / mf, g("SQ_INSTS_SALU") / mf,
               g("SQ_INSTS_LDS") / mf, g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"),
               g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"),
               g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))]
        print(f"| {tag} | `{', '.join(sorted(names))[:60]}` | " + " | ".join(f"{v:.3f}" for v in row) + " |")


if __name__ == "__main__":
    main()

"""Per-layer counters of Inception-v3's convs (BASELINE config 5): for every
unique conv of scripts/conv_layers.py's --json output, two rocprofv3 --pmc
passes (each its own run) of that layer alone on the tile the autotuner
picked (TFA_GEMM_TILE), then one markdown table: ms, TF/s, tile, MFMA busy,
VALU per MFMA, LDS bank conflicts, wait shares (definitions as
scripts/pmc_summary.py). This driver never touches the GPU itself: each pass
is `rocprofv3 ... -- python3 scripts/conv_layers.py --only i`.

    python scripts/conv_layers.py --json L.json && python scripts/layers_pmc.py --layers L.json --out DIR
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PA = ("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY "
      "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE")
PB = ("SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU "
      "SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE")


def counters(d):
    agg = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "tfa::k::" in n and "fill" not in n and "pool" not in n:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--last", type=int, default=10 ** 9)
    ap.add_argument("--table-only", action="store_true", help="only rebuild the table from layers_pmc_*.json")
    a = ap.parse_args()
    layers = [L for L in json.load(open(a.layers))["layers"] if a.first <= L["index"] <= a.last]
    os.makedirs(a.out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    rows = []
    for L in ([] if a.table_only else layers):
        i = L["index"]
        e = dict(env)
        if isinstance(L.get("tile"), int):
            e["TFA_GEMM_TILE"] = str(L["tile"])
        res = {}
        for tag, pmc in (("a", PA), ("b", PB)):
            d = os.path.join(a.out, f"l{i}{tag}")
            cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *pmc.split(), "--output-format", "csv",
                   "-d", d, "-o", "run", "--", sys.executable, "scripts/conv_layers.py", "--only", str(i),
                   "--iters", "2", "--batch", str(a.batch)]
            p = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True)
            if p.returncode != 0:
                print(f"layer {i} pass {tag} rc={p.returncode}: {p.stderr[-800:]}", flush=True)
                sys.exit(1)
            res.update(counters(d))
        mf = max(res.get("SQ_INSTS_MFMA", 0.0), 1.0)
        busy = res.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1024 * res.get("GRBM_GUI_ACTIVE", 1.0) / 8, 1.0)
        wave = max(res.get("SQ_WAVE_CYCLES", 1.0), 1.0)
        row = dict(L, mfma_busy=busy, valu_per_mfma=(res.get("SQ_INSTS_VALU", 0.0) - mf) / mf,
                   lds_conflict=res.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(res.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0),
                   wait_any=res.get("SQ_WAIT_ANY", 0.0) / wave, salu_per_mfma=res.get("SQ_INSTS_SALU", 0.0) / mf)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if rows:
        with open(os.path.join(a.out, f"layers_pmc_{a.first}.json"), "w") as f:
            json.dump(rows, f, indent=1)
    rows = sorted((r for p in glob.glob(os.path.join(a.out, "layers_pmc_*.json")) for r in json.load(open(p))),
                  key=lambda r: r["index"])
    tot = sum(r["ms"] * r["count"] for r in json.load(open(a.layers))["layers"])
    lines = ["| # | layer | x | shape | M | K | OC | tile | ms | share | TF/s | MFMA busy | VALU/MFMA | SALU/MFMA | LDS confl. | wait_any |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        shape = f"{r['H']}x{r['W']}x{r['C']} k{r['KH']}x{r['KW']} s{r['stride']} {r['pad']}"
        tile = f"{r['tile']} ({r.get('tile_dims')}, {r.get('core')})" if r.get("tile") is not None else "direct"
        lines.append(f"| {r['index']} | {r['layer']} | {r['count']} | {shape} | {r['M']} | {r['K']} | {r['OC']} | {tile} | "
                     f"{r['ms']:.3f} | {100 * r['ms'] * r['count'] / tot:.1f}% | {r['tflops']:.1f} | {r['mfma_busy']:.3f} | "
                     f"{r['valu_per_mfma']:.2f} | {r['salu_per_mfma']:.2f} | {r['lds_conflict']:.3f} | {r['wait_any']:.3f} |")
    with open(os.path.join(a.out, "layers_pmc.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()

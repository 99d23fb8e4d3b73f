"""Build the shipped gfx950 default tile table (tensorframes_amd/tiles/gfx950.json)
from the BASELINE workloads as the engine plans them: the headline bench
(10M x 512 x 512 MatMul chunks) and Inception-v3 device-resident scoring
(every conv, with its fused sibling segments). Each runs in its own process
with TFA_GEMM_TUNE_DUMP, which merges that process's autotuner picks into the
table at exit; run it on the GPU box, then commit the JSON.

    python scripts/tile_table.py [--out tensorframes_amd/tiles/gfx950.json]
    python scripts/tile_table.py --add-read-image   # keep every entry, add the VGG-16
                                                    # read_image shapes (FC GEMMs)
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tensorframes_amd", "tiles", "gfx950.json"))
    ap.add_argument("--add-read-image", action="store_true",
                    help="merge the shapes of examples/read_image.py (VGG-16 scoring) into the existing table, "
                         "tuned with the table's defaults in force (a default moves only on a 2%% win, twice)")
    a = ap.parse_args()
    a.out = os.path.abspath(a.out)
    if a.add_read_image:
        import shutil
        tmp = a.out + ".new"
        shutil.copyfile(os.path.join(REPO, "tensorframes_amd", "tiles", "gfx950.json"), tmp)  # the shipped table
        before = len(json.load(open(tmp))["entries"])
        env = dict(os.environ, TFA_GEMM_TUNE_DUMP=tmp)
        r = subprocess.run([sys.executable, "examples/read_image.py", "--images", "2048"], cwd=REPO, env=env,
                           timeout=900)
        if r.returncode != 0:
            sys.exit(r.returncode)
        table = json.load(open(tmp))
        table["note"] = table.get("note", "") + "; plus the autotuner picks of examples/read_image.py (VGG-16)"
        with open(a.out, "w") as f:
            json.dump(table, f, indent=1)
        os.remove(tmp)
        print(f"{before} -> {len(table['entries'])} entries -> {a.out}")
        return
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    tmp = a.out + ".new"
    if os.path.exists(tmp):
        os.remove(tmp)
    # no defaults while measuring: every shape is tuned from scratch
    env = dict(os.environ, TFA_GEMM_TUNE_DUMP=tmp, TFA_GEMM_DEFAULTS="0")
    runs = [[sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--mode", "device"],
            [sys.executable, "bench/configs.py", "inception", "--source", "device", "--rows", "4096", "--steps", "1",
             "--warmup", "1"]]
    for cmd in runs:
        print("==", " ".join(cmd[1:]), flush=True)
        r = subprocess.run(cmd, cwd=REPO, env=env, timeout=900)
        if r.returncode != 0:
            sys.exit(r.returncode)
    with open(tmp) as f:
        table = json.load(f)
    table["note"] = ("autotuner picks of bench.py (device) and bench/configs.py inception (device) on one "
                     "MI355X; key = (M, N, K, batch, A loader, B^T, vec, conv H, W, C, KW, OH, OW, sh, sw, dh, dw, "
                     "pt, pl, ldc==N + 2 * fused segments)")
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1)
    os.remove(tmp)
    print(f"{len(table['entries'])} entries -> {a.out}")


if __name__ == "__main__":
    main()

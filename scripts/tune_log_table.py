"""Table of the GEMM autotuner's candidate timings (TFA_GEMM_TUNE_LOG=1 lines
on stderr, "[gemm tune] M=.. N=.. K=.. ... best=.. | tile:ms ..."): per shape,
the fastest round-4-core tile and the fastest g2-core tile, which one the
tuner kept and by how much the other loses. The evidence for the shapes that
stay on round-4 tiles (round-5 verdict: "move them to g2 or explain why g2
loses there").

    TFA_GEMM_TUNE_LOG=1 python bench/configs.py inception ... 2> tune.log
    python scripts/tune_log_table.py tune.log > profiles/r6_layers/tile_choice.md
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorframes_amd._native import _C  # noqa: E402

LINE = re.compile(r"\[gemm tune\] M=(\d+) N=(\d+) K=(\d+) al=(\d+) conv=(\d+)x(\d+)x(\d+) heur=(-?\d+) "
                  r"default=(-?\d+)( \(replaced\))? best=(-?\d+) \|(.*)")


def main():
    first_g2 = next(i for i in range(_C.gemm_tile_count()) if _C.gemm_tile_dims(i)[2] == 2)
    name = lambda t: "{}x{}".format(*_C.gemm_tile_dims(t)[:2])  # noqa: E731
    rows = []
    for line in open(sys.argv[1]):
        m = LINE.search(line)
        if not m:
            continue
        M, N, K, al, H, W, C = (int(m.group(i)) for i in range(1, 8))
        best = int(m.group(11))
        cand = {int(a): float(b) for a, b in (kv.split(":") for kv in m.group(12).split())}
        r4 = {t: v for t, v in cand.items() if t < first_g2}
        g2 = {t: v for t, v in cand.items() if t >= first_g2}
        br4 = min(r4, key=r4.get) if r4 else None
        bg2 = min(g2, key=g2.get) if g2 else None
        rows.append((M, N, K, "conv %dx%dx%d" % (H, W, C) if H else "gemm", best, br4, bg2, r4.get(br4), g2.get(bg2),
                     m.group(10) is not None))
    print("| M | N | K | A | kept | best round-4 tile (ms) | best g2 tile (ms) | g2 vs round-4 |")
    print("|---:|---:|---:|---|---|---|---|---:|")
    for M, N, K, kind, best, br4, bg2, t4, tg, repl in rows:
        core = "g2" if best >= first_g2 else "round-4"
        rel = f"{(tg / t4 - 1) * 100:+.1f} %" if t4 and tg else ""
        print(f"| {M} | {N} | {K} | {kind} | {core} {name(best)}{' (replaced the default)' if repl else ''} | "
              f"{name(br4) if br4 is not None else '-'} ({t4:.4f}) | "
              f"{name(bg2) if bg2 is not None else '-'} ({tg if tg else float('nan'):.4f}) | {rel} |")


if __name__ == "__main__":
    main()

"""Per-key harmonic mean: map_blocks -> aggregate -> map_blocks (reference:
src/main/python/tensorframes_snippets/geom_mean.py).

    python examples/harmonic_mean.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import Row  # noqa: E402
from tensorframes_amd.models.harmonic_mean import harmonic_mean  # noqa: E402


def main():
    df = tfs.create_dataframe([Row(key=k, x=float(v)) for k, v in
                               [("a", 1), ("a", 2), ("a", 4), ("b", 3), ("b", 6)]])
    for r in sorted(harmonic_mean(df).collect()):
        print(r)


if __name__ == "__main__":
    main()

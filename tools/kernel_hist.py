#!/usr/bin/env python
"""Per-dispatch duration histogram of selected kernels from a rocprofv3 kernel trace
(the SQLite ``.db`` or a ``*kernel_trace.csv``; a directory is searched for either).

usage: python tools/kernel_hist.py <trace.db | kernel_trace.csv | dir> <substring> [...]
"""
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnmf_torch_amd.profiling import _load  # noqa: E402


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True)) + \
            sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))
        path = found[0]
    df = _load(path)
    edges = [0, 10, 50, 100, 200, 400, 800, 1600, 1e9]
    for s in sys.argv[2:]:
        d = df[df["name"].str.contains(s, regex=False)]["dur"].to_numpy() / 1e3
        if d.size == 0:
            print(f"{s}: none")
            continue
        h, _ = np.histogram(d, bins=edges)
        print(f"{s}: n={d.size} sum={d.sum() / 1e3:.1f} ms  p50={np.median(d):.1f}us "
              f"p90={np.percentile(d, 90):.1f}us max={d.max():.1f}us")
        for a, b, c in zip(edges[:-1], edges[1:], h):
            t = float(d[(d >= a) & (d < b)].sum()) / 1e3
            print(f"   [{a:>6.0f}, {b:>6.0f}) us: {c:6d} dispatches, {t:8.1f} ms")


if __name__ == "__main__":
    main()

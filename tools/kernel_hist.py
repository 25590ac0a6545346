#!/usr/bin/env python
"""Per-dispatch duration histogram of selected kernels from a rocprofv3 kernel-trace CSV
(find it under the -d directory: ``*_kernel_trace.csv``).

usage: python tools/kernel_hist.py <kernel_trace.csv> <substring> [<substring> ...]
"""
import csv
import glob
import os
import sys

import numpy as np


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    subs = sys.argv[2:]
    durs = {s: [] for s in subs}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            for s in subs:
                if s in name:
                    durs[s].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    edges = [0, 10, 50, 100, 200, 400, 800, 1600, 1e9]
    for s, d in durs.items():
        d = np.asarray(d)
        if d.size == 0:
            print(f"{s}: none")
            continue
        h, _ = np.histogram(d, bins=edges)
        tot = [float(d[(d >= a) & (d < b)].sum()) / 1e3 for a, b in zip(edges[:-1], edges[1:])]
        print(f"{s}: n={d.size} sum={d.sum() / 1e3:.1f} ms  p50={np.median(d):.1f}us "
              f"p90={np.percentile(d, 90):.1f}us max={d.max():.1f}us")
        for a, b, c, t in zip(edges[:-1], edges[1:], h, tot):
            print(f"   [{a:>6.0f}, {b:>6.0f}) us: {c:6d} dispatches, {t:8.1f} ms")


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Per-kernel mean of rocprofv3 --pmc counter values (counter_collection.csv files).

usage: python tools/pmc_summary.py <dir with */run_counter_collection.csv> [--top N]
"""
import argparse
import glob
import os
import re

import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    out = []
    for f in sorted(glob.glob(os.path.join(a.root, "*", "run_counter_collection.csv"))):
        df = pd.read_csv(f)
        tag = os.path.basename(os.path.dirname(f))
        df["kernel"] = df["Kernel_Name"].map(lambda n: re.sub(r"\(.*", "", n)[:70])
        g = df.groupby(["kernel", "Counter_Name"])["Counter_Value"].agg(["count", "mean"])
        g = g.reset_index().sort_values("count", ascending=False)
        out.append(f"== {tag}")
        out.append(g.head(a.top).to_string(index=False, float_format=lambda v: f"{v:.2f}"))
    print("\n".join(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""GPU idle gaps between consecutive kernels of a rocprofv3 kernel trace (.db or
kernel_trace.csv): total busy / idle time and the largest gaps with the kernels around
them -- where the host (launch latency, synchronisation) leaves the GPU idle.

usage: python tools/gap_summary.py <trace.db | kernel_trace.csv> [--min-us 5] [--top 15]
"""
import argparse
import os
import re
import sqlite3
import sys

import pandas as pd


def load(path):
    if path.endswith(".csv"):
        df = pd.read_csv(path)
        return pd.DataFrame({"name": df["Kernel_Name"], "start": df["Start_Timestamp"],
                             "end": df["End_Timestamp"]})
    con = sqlite3.connect(path)
    df = pd.read_sql_query("select * from kernels", con)
    name_col = "kernel_name" if "kernel_name" in df.columns else "name"
    return pd.DataFrame({"name": df[name_col], "start": df["start"], "end": df["end"]})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--from-frac", type=float, default=0.0,
                    help="only the trace after this fraction of its span (skip warmup)")
    a = ap.parse_args()
    df = load(a.path).sort_values("start").reset_index(drop=True)
    t0, t1 = df["start"].min(), df["end"].max()
    df = df[df["start"] >= t0 + a.from_frac * (t1 - t0)].reset_index(drop=True)
    df["short"] = df["name"].map(lambda n: re.sub(r"\(.*", "", n)[:60])
    ends = df["end"].cummax().shift(1)
    gap = (df["start"] - ends).fillna(0).clip(lower=0) / 1e3
    span = (df["end"].max() - df["start"].min()) / 1e3
    busy = span - gap.sum()
    big = gap[gap >= a.min_us]
    print(f"span {span / 1e3:.2f} ms, idle {gap.sum() / 1e3:.2f} ms ({100 * gap.sum() / span:.1f} %), "
          f"{len(big)} gaps >= {a.min_us} us totalling {big.sum() / 1e3:.2f} ms")
    prev = df["short"].shift(1)
    pairs = pd.DataFrame({"gap_us": gap, "after": prev, "before": df["short"]})
    agg = pairs[pairs.gap_us >= a.min_us].groupby(["after", "before"])["gap_us"].agg(
        ["count", "sum", "mean"]).sort_values("sum", ascending=False)
    print(agg.head(a.top).to_string(float_format=lambda v: f"{v:.1f}"))


if __name__ == "__main__":
    sys.exit(main())

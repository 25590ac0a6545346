#!/usr/bin/env python
"""Summarise a rocprofv3 SQLite (.db) or kernel-trace CSV into a per-kernel table.

usage: python tools/prof_summary.py <run_results.db | kernel_trace.csv> [--top N]
"""
import argparse
import re
import sqlite3
import sys

import pandas as pd


def load(path):
    if path.endswith(".csv"):
        df = pd.read_csv(path)
        name = "Kernel_Name"
        df["dur"] = df["End_Timestamp"] - df["Start_Timestamp"]
        return df.rename(columns={name: "name"})[["name", "dur"]]
    con = sqlite3.connect(path)
    df = pd.read_sql_query("select * from kernels", con)
    name_col = "kernel_name" if "kernel_name" in df.columns else "name"
    df["dur"] = df["end"] - df["start"]
    return df.rename(columns={name_col: "name"})[["name", "dur"]]


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    df = load(a.path)
    df["kernel"] = df["name"].map(short)
    g = df.groupby("kernel")["dur"].agg(["count", "sum", "mean"]).sort_values("sum", ascending=False)
    tot = g["sum"].sum()
    g["pct"] = 100 * g["sum"] / tot
    g["sum_ms"] = g["sum"] / 1e6
    g["mean_us"] = g["mean"] / 1e3
    print(f"total kernel time: {tot/1e6:.3f} ms over {int(g['count'].sum())} dispatches")
    print(g[["count", "sum_ms", "mean_us", "pct"]].head(a.top).to_string(float_format=lambda v: f"{v:.3f}"))


if __name__ == "__main__":
    sys.exit(main())

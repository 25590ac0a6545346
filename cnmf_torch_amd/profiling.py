"""Kernel-level profiling of any cnmf stage (SURVEY.md §5.1 "--profile mode").

    python -m cnmf_torch_amd.profiling --out prof_dir -- factorize --output-dir out --name run
    python -m cnmf_torch_amd.profiling --out prof_dir --pmc SQ_INSTS_VALU,SQ_INSTS_MFMA -- ...

Runs ``rocprofv3 --kernel-trace --stats`` (or a counter collection with ``--pmc``; the two
are never combined with API/runtime tracing) around ``python -m cnmf_torch_amd <args>`` as
a CHILD process -- the profiler's preload initialises the GPU, so this process never
execs -- then writes ``<out>/kernel_summary.txt``: per-kernel dispatch count, total and
mean time, share of GPU time.  ``summarize`` also reads existing trace CSVs / SQLite DBs.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import shutil
import sqlite3
import subprocess
import sys


def _load(path: str):
    import pandas as pd

    if path.endswith(".csv"):
        df = pd.read_csv(path)
        df["dur"] = df["End_Timestamp"] - df["Start_Timestamp"]
        return df.rename(columns={"Kernel_Name": "name"})[["name", "dur"]]
    con = sqlite3.connect(path)
    df = pd.read_sql_query("select * from kernels", con)
    name_col = "kernel_name" if "kernel_name" in df.columns else "name"
    df["dur"] = df["end"] - df["start"]
    return df.rename(columns={name_col: "name"})[["name", "dur"]]


def summarize(path: str, top: int = 30) -> str:
    """Per-kernel table of a rocprofv3 kernel-trace CSV or SQLite database."""
    df = _load(path)
    df["kernel"] = df["name"].map(lambda n: re.sub(r"\(.*", "", n)[:110])
    g = df.groupby("kernel")["dur"].agg(["count", "sum", "mean"]).sort_values("sum",
                                                                           ascending=False)
    tot = g["sum"].sum()
    g["pct"] = 100 * g["sum"] / tot
    g["sum_ms"] = g["sum"] / 1e6
    g["mean_us"] = g["mean"] / 1e3
    head = f"total kernel time: {tot / 1e6:.3f} ms over {int(g['count'].sum())} dispatches\n"
    return head + g[["count", "sum_ms", "mean_us", "pct"]].head(top).to_string(
        float_format=lambda v: f"{v:.3f}")


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        print(__doc__)
        return 2
    cut = argv.index("--")
    ap = argparse.ArgumentParser(prog="python -m cnmf_torch_amd.profiling")
    ap.add_argument("--out", default="cnmf_profile")
    ap.add_argument("--pmc", default=None, help="comma-separated hardware counters")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv[:cut])
    cmd_args = argv[cut + 1:]
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    os.makedirs(a.out, exist_ok=True)
    cmd = [prof, "-d", a.out, "-o", "run", "--output-format", "csv"]
    if a.pmc:
        cmd += ["--pmc"] + a.pmc.split(",")
    else:
        cmd += ["--kernel-trace", "--stats"]
    cmd += ["--", sys.executable, "-m", "cnmf_torch_amd"] + cmd_args
    print(" ".join(cmd), flush=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    rc = subprocess.call(cmd, env=env)
    traces = sorted(glob.glob(os.path.join(a.out, "**", "*kernel_trace.csv"), recursive=True))
    if traces and not a.pmc:
        text = summarize(traces[-1], a.top)
        with open(os.path.join(a.out, "kernel_summary.txt"), "w") as fh:
            fh.write(text + "\n")
        print(text)
    return rc


if __name__ == "__main__":
    sys.exit(main())

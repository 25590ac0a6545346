#!/usr/bin/env python
"""Summarise a rocprofv3 SQLite (.db) or kernel-trace CSV into a per-kernel table.

usage: python tools/prof_summary.py <run_results.db | kernel_trace.csv> [--top N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnmf_torch_amd.profiling import summarize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    print(summarize(a.path, a.top))


if __name__ == "__main__":
    sys.exit(main())

"""Per-pass breakdown of a rocprofv3 kernel trace of bench.py (rocpd SQLite output).

Passes end at ``conv_update_kernel`` (one per online pass, csrc/kernels/conv.hip).  For
each pass of the last ``--runs`` factorisation runs it prints the GPU-busy time (sum of
kernel durations), the pass wall (first start to last end), the idle gap, the number of
dispatches, and the busy time per kernel family -- which says whether a pass is bound by
kernel time or by the gaps between launches (host enqueue).

    python tools/trace_passes.py gpurun_out/r3a/prof/run_results.db [--runs 1]
"""
import argparse
import collections
import re
import sqlite3


def family(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    for key in ("solve_pipe_kernel", "solve_mfma_kernel", "gemm_planes_kernel", "gemm_reduce",
                "gram_reduce", "gram_kernel", "conv_update", "split_planes", "bp_", "beta_"):
        if key in n:
            return key
    return n.split("<")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--runs", type=int, default=1, help="last N runs (a run starts at init)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y from kernels order by start").fetchall()
    # a factorisation run begins with philox_fill (Philox init of H, W)
    starts = [i for i, r in enumerate(rows) if "philox_fill" in r[0]]
    run_starts = []
    for i in starts:       # two philox launches per run (H, W): keep the first of each pair
        if not run_starts or i - run_starts[-1] > 4:
            run_starts.append(i)
    sel = rows[run_starts[-a.runs]:] if len(run_starts) >= a.runs else rows
    passes, cur = [], []
    for r in sel:
        cur.append(r)
        if "conv_update" in r[0]:
            passes.append(cur)
            cur = []
    tot_busy = tot_wall = 0.0
    print(f"{'pass':>4} {'disp':>5} {'busy_us':>9} {'wall_us':>9} {'idle_us':>8}  top families (us)")
    for p, ks in enumerate(passes):
        busy = sum((e - s) for _, s, e, _, _ in ks) / 1e3
        wall = (ks[-1][2] - ks[0][1]) / 1e3
        fam = collections.Counter()
        for n, s, e, _, _ in ks:
            fam[family(n)] += (e - s) / 1e3
        top = ", ".join(f"{k} {v:.0f}" for k, v in fam.most_common(5))
        solve_grid = [gx for n, _, _, gx, _ in ks if "solve" in n][:1]
        print(f"{p:>4} {len(ks):>5} {busy:>9.1f} {wall:>9.1f} {wall - busy:>8.1f}  "
              f"[R~{solve_grid[0] if solve_grid else '-'}] {top}")
        tot_busy += busy
        tot_wall += wall
    print(f"total: busy {tot_busy / 1e3:.3f} ms, pass wall {tot_wall / 1e3:.3f} ms, "
          f"{len(passes)} passes")
    fam = collections.Counter()
    cnt = collections.Counter()
    for n, s, e, _, _ in sel:
        fam[family(n)] += (e - s) / 1e3
        cnt[family(n)] += 1
    for k, v in fam.most_common(12):
        print(f"  {k:<40} {v:9.1f} us  {cnt[k]:5d} calls")


if __name__ == "__main__":
    main()

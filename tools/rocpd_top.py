"""Top-N kernel summary (name, calls, total ms, mean us, %) from a rocprofv3 results
database (rocpd SQLite, the default output of rocprofv3 --kernel-trace --stats in ROCm 7).

    python tools/rocpd_top.py gpurun_out/x/prof/hs_results.db [N] > profiles/x.txt
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    tot = sum(r[2] for r in rows)
    print(f"# {db}: {len(rows)} kernels, {sum(r[1] for r in rows)} dispatches, "
          f"{tot / 1e3:.3f} ms GPU total (rocpd top_kernels durations are in us)")
    print(f"{'calls':>7} {'total_ms':>10} {'mean_us':>10} {'pct':>6}  name")
    for name, calls, total, avg, pct in rows[:n]:
        nm = name if len(name) < 140 else name[:137] + "..."
        print(f"{calls:7d} {total / 1e3:10.3f} {avg:10.2f} {pct:6.2f}  {nm}")
    cijk = [r for r in rows if r[0].startswith("Cijk")]
    print(f"# library GEMM (Cijk_*) kernels: {len(cijk)}")


if __name__ == "__main__":
    main()

"""Phase breakdown of the pipelined MU solve (csrc/kernels/solve_pipe.h) from in-kernel
s_memtime stamps (diagnostic only: ops.STAMPS_ON gives each launch a stamp buffer
that nothing else reads).  Runs one bench-shaped factorisation (graphs off, so every pass
is an eager, stamped launch) and prints, per K and side (slice count), the mean cycles per
workgroup in: prologue (operand loads, slab / partial-Gram sums), the sweep loop minus
the objective checks, the checks (objective chain + block reduce + cooperative exchange),
and the epilogue (stores, planes, partial Gram), plus the launch span (first start to
last end) against the mean workgroup time -- the load-imbalance tail.

    CNMF_GRAPHS=0 python tools/pipe_stamp_probe.py --k 20

The stamps exist only in a probe build of the extension: build with
``CNMF_PIPE_STAMPS_BUILD=1 python -c "import cnmf_torch_amd._build as b; b.build_hip()"``
(and rebuild without it afterwards: the production kernels carry no stamp code).
"""
import argparse
import json
import os
import sys

os.environ.setdefault("CNMF_GRAPHS", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd import ops  # noqa: E402

ops.STAMPS_ON = True
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--genes", type=int, default=2000)
    a = ap.parse_args()
    X = torch.from_numpy(normalized_counts_matrix(a.cells, a.genes, n_programs=a.k, seed=0)).cuda()
    opts = NMFOptions(n_components=a.k, tol=1e-4, online_chunk_size=5000,
                      online_chunk_max_iter=1000)
    solver = NMFBatchSolver(X, opts)
    np.random.seed(14)
    seeds = [int(s) for s in np.random.randint(1, 2 ** 31 - 1, size=a.reps)]
    solver.run(seeds)            # warm-up (module loads, plans)
    ops.STAMP_LOG.clear()
    solver.run(seeds)
    torch.cuda.synchronize()
    groups = {}
    for e in ops.STAMP_LOG:
        s3 = e["buf"].view(-1, 10).cpu().numpy().astype(np.int64)
        S = max(1, int(e["S"]))
        # start skew among the slices of one replicate (buffer is slice-major: slice *
        # blocks + block), in us of the 100 MHz realtime counter
        skew, askew = [], []
        if S > 1 and s3.shape[0] % S == 0:
            v = s3.reshape(S, -1, 10)
            ran = (v[:, :, 1] > 0).all(axis=0)
            if ran.any():
                st = v[:, ran, 0]
                skew = list((st.max(axis=0) - st.min(axis=0)) * 0.01)
                # arrival spread at the first cooperative exchange (realtime, us)
                ax = v[:, ran, 6]
                ok = (ax > 0).all(axis=0)
                if ok.any():
                    askew = list((ax[:, ok].max(axis=0) - ax[:, ok].min(axis=0)) * 0.01)
        s = s3[s3[:, 1] > 0]                     # workgroups that ran (active replicates)
        if s.size == 0:
            continue
        key = (e["K"], e["S"])
        g = groups.setdefault(key, {"launches": 0, "pro": [], "loop": [], "chk": [], "epi": [],
                                    "wg": [], "span": [], "sweeps": [], "checks": [],
                                    "skew": [], "askew": []})
        g["skew"].extend(skew)
        g["askew"].extend(askew)
        # workgroups per CU of this launch: (XCD, SE, SH, CU) from HW_ID / XCC_ID
        hw = s[:, 8]
        cu = (s[:, 9] & 0xF) * 4096 + ((hw >> 13) & 0x7) * 512 + ((hw >> 12) & 1) * 256 + \
            ((hw >> 8) & 0xF)
        _, per_cu = np.unique(cu, return_counts=True)
        g.setdefault("cus", []).append(len(per_cu))
        g.setdefault("wpc_max", []).append(int(per_cu.max()))
        g.setdefault("wpc_mean", []).append(float(per_cu.mean()))
        g.setdefault("wgs", []).append(int(s.shape[0]))
        g["launches"] += 1
        g["pro"].append(np.mean(s[:, 2]))
        g["chk"].append(np.mean(s[:, 4]))
        g["loop"].append(np.mean(s[:, 3] - s[:, 4]))
        g["epi"].append(np.mean(s[:, 5]))
        g["wg"].append(np.mean(s[:, 1] - s[:, 0]) * 0.01)            # us (100 MHz)
        g["span"].append(float(s[:, 1].max() - s[:, 0].min()) * 0.01)  # us
        g["sweeps"].append(np.mean(s[:, 7] & 0xffffffff))
        g["checks"].append(np.mean(s[:, 7] >> 32))
    if not groups:
        sys.exit("no stamps were written: build the extension with CNMF_PIPE_STAMPS_BUILD=1")
    for (K, S), g in sorted(groups.items()):
        print(json.dumps({
            "K": K, "slices": S, "launches": g["launches"],
            "cycles_per_wg": {k: round(float(np.mean(g[k])), 0)
                              for k in ("pro", "loop", "chk", "epi")},
            "wg_us": round(float(np.mean(g["wg"])), 2),
            "launch_span_us": round(float(np.mean(g["span"])), 2),
            "mean_sweeps": round(float(np.mean(g["sweeps"])), 2),
            "mean_checks": round(float(np.mean(g["checks"])), 2),
            "slice_start_skew_us": (round(float(np.mean(g["skew"])), 2) if g["skew"] else None),
            "slice_start_skew_p90_us": (round(float(np.percentile(g["skew"], 90)), 2)
                                        if g["skew"] else None),
            "wgs": round(float(np.mean(g["wgs"])), 1),
            "cus_used": round(float(np.mean(g["cus"])), 1),
            "wg_per_cu_mean": round(float(np.mean(g["wpc_mean"])), 2),
            "wg_per_cu_max": round(float(np.mean(g["wpc_max"])), 2),
            "first_exchange_arrival_spread_us": (round(float(np.mean(g["askew"])), 2)
                                                 if g["askew"] else None),
            "first_exchange_arrival_spread_p90_us": (
                round(float(np.percentile(g["askew"], 90)), 2) if g["askew"] else None)}),
            flush=True)


if __name__ == "__main__":
    main()

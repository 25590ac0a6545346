"""The Harmony clustering + PC ridge loop alone (models/harmony.py run_harmony) on
synthetic PCs -- for kernel summaries of the Harmony stage without the preprocessing and
cNMF launches around it (tools/bench_harmony.py times the whole config-5 pipeline).

    rocprofv3 --kernel-trace --stats -d gpurun_out/hs -- python tools/harmony_stage.py

Synthetic PCs: 12 cell types in 50 dimensions, additive shifts for 4 categorical
covariates with (6, 4, 3, 2) levels, Gaussian noise.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd.models.harmony import run_harmony  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=500000)
    ap.add_argument("--pcs", type=int, default=50)
    ap.add_argument("--max-iter-harmony", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=1, help="timed runs after one warm-up run")
    a = ap.parse_args()
    rs = np.random.default_rng(0)
    n, d = a.cells, a.pcs
    levels = (6, 4, 3, 2)
    types = rs.integers(0, 12, n)
    Z = rs.normal(size=(12, d))[types] * 3.0
    cov = {}
    for i, L in enumerate(levels):
        lab = rs.integers(0, L, n)
        Z += rs.normal(size=(L, d))[lab] * 1.5
        cov[f"cov{i}"] = pd.Categorical([f"c{i}_{v}" for v in range(L)])[lab]
    Z += rs.normal(size=(n, d))
    meta = pd.DataFrame(cov)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    kw = dict(max_iter_harmony=a.max_iter_harmony, random_state=0, device=dev,
              init_backend="device" if dev == "cuda" else "sklearn")
    res = run_harmony(Z, meta, list(cov), **kw)           # warm-up (code objects, caches)
    times = []
    for _ in range(a.repeat):
        if dev == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = run_harmony(Z, meta, list(cov), **kw)
        if dev == "cuda":
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    print(json.dumps({"metric": "Harmony stage wall-clock (run_harmony on PCs)", "unit": "s",
                      "value": round(min(times), 3), "runs_s": [round(t, 3) for t in times],
                      "iterations": len(res.kmeans_rounds),
                      "kmeans_rounds": [int(r) + 1 for r in res.kmeans_rounds],
                      "K": int(res.K),
                      "config": {"cells": n, "pcs": d, "covariates": levels,
                                 "max_iter_harmony": a.max_iter_harmony, "device": dev},
                      "data": "synthetic PCs: 12 types + 4 additive covariate shifts + noise"}))


if __name__ == "__main__":
    main()

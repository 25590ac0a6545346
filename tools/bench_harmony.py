"""Harmony batch correction + cNMF end to end (BASELINE.json config 5: 500k cells,
4 batch covariates).

    python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000

Simulates sparse counts from planted programs with multiplicative per-gene effects for
four categorical covariates, then times:

1. Preprocess.preprocess_for_cnmf(harmony_vars=[4 covariates]) with the stages
   normalise -> seurat_v3 HVG -> scale/ceiling -> PCA -> Harmony -> MOE ridge correction;
   Harmony's R-update runs in the fused HIP kernels.
2. cNMF prepare -> factorize (K=10, --n-iter replicates) -> combine -> consensus on the
   corrected matrix.

Prints one JSON line with the stage wall-clocks.
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd import Preprocess, cNMF  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402


def _sim_part(args):
    S, effects, covs, seed, a, b, programs = args
    # one generator per row block: the matrix does not depend on the worker count
    r = np.random.default_rng([seed, a])
    U = r.dirichlet(np.full(programs, 0.3), b - a)
    lib = r.lognormal(np.log(1500.0), 0.35, b - a)
    lam = (U @ S) * lib[:, None]
    for i, e in enumerate(effects):
        lam *= e[covs[i]]
    x = r.poisson(lam)
    m = x != 0
    return (np.cumsum(m.sum(axis=1)), np.nonzero(m)[1].astype(np.int32),
            x[m].astype(np.float32))


def simulate(n, g, programs=8, n_cov=4, levels=(6, 4, 3, 2), seed=0, block=2500):
    rs = np.random.default_rng(seed)
    base = rs.lognormal(0.0, 1.0, g)
    S = np.tile(base, (programs, 1))
    for k in range(programs):
        idx = rs.choice(g, int(0.15 * g), replace=False)
        S[k, idx] *= rs.lognormal(1.5, 0.5, idx.size)
    S /= S.sum(1, keepdims=True)
    covs = {f"cov{i}": rs.integers(0, levels[i], n) for i in range(n_cov)}
    effects = [rs.lognormal(0.0, 0.3, (levels[i], g)) for i in range(n_cov)]
    jobs = [(S, effects, [covs[f"cov{i}"][a:min(n, a + block)] for i in range(n_cov)], seed,
             a, min(n, a + block), programs) for a in range(0, n, block)]
    import multiprocessing as mp
    with mp.get_context("fork").Pool(min(16, os.cpu_count() or 1, len(jobs))) as pool:
        parts = pool.map(_sim_part, jobs)
    ptr = [np.zeros(1, dtype=np.int64)]
    base = 0
    for c, _, _ in parts:
        ptr.append(c + base)
        base += int(c[-1]) if c.size else 0
    X = sp.csr_matrix((np.concatenate([p[2] for p in parts]),
                       np.concatenate([p[1] for p in parts]), np.concatenate(ptr)), shape=(n, g))
    obs = pd.DataFrame({k: pd.Categorical([f"{k}_{v}" for v in val]) for k, val in covs.items()},
                       index=[f"c{i}" for i in range(n)])
    return AnnData(X=X, obs=obs, var=pd.DataFrame(index=[f"g{j}" for j in range(g)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=500000)
    ap.add_argument("--genes", type=int, default=3000)
    ap.add_argument("--hvg", type=int, default=2000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iter", type=int, default=100)
    ap.add_argument("--max-iter-harmony", type=int, default=20,
                    help="the reference default (preprocess.py:138)")
    ap.add_argument("--gpu-busy", action="store_true",
                    help="also report GPU-busy seconds per stage (torch.profiler kernel time; "
                         "adds profiler overhead to the wall-clocks)")
    ap.add_argument("--profile", default=None, help="cProfile the Harmony stage into this file")
    ap.add_argument("--profile-stages", default=None,
                    help="cProfile prepare / factorize / combine+consensus into PREFIX.<stage>.txt")
    a = ap.parse_args()

    busy = {}

    def staged(name, fn):
        if a.gpu_busy and torch.cuda.is_available():
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CUDA]) as pr:
                out = fn()
                torch.cuda.synchronize()
            busy[name] = round(sum(e.self_device_time_total for e in pr.key_averages()) / 1e6, 3)
            return out
        if not a.profile_stages:
            return fn()
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        try:
            return fn()
        finally:
            pr.disable()
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(45)
            with open(f"{a.profile_stages}.{name}.txt", "w") as fh:
                fh.write(buf.getvalue())
    t = {}
    t0 = time.perf_counter()
    ad = simulate(a.cells, a.genes)
    t["simulate"] = time.perf_counter() - t0
    work = tempfile.mkdtemp(prefix="cnmf_harmony_")
    base = os.path.join(work, "hm")
    p = Preprocess(random_seed=0)
    t0 = time.perf_counter()
    prof = None
    if a.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    corrected, tp10k, hvgs = staged("preprocess_harmony", lambda: p.preprocess_for_cnmf(
        ad, harmony_vars=["cov0", "cov1", "cov2", "cov3"], n_top_rna_genes=a.hvg,
        makeplots=False, max_iter_harmony=a.max_iter_harmony, save_output_base=base))
    if prof is not None:
        import io
        import pstats
        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(40)
        with open(a.profile, "w") as fh:
            fh.write(buf.getvalue())
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    t["preprocess_harmony"] = time.perf_counter() - t0
    obj = cNMF(output_dir=work, name="hm_cnmf")
    t0 = time.perf_counter()
    staged("prepare", lambda: obj.prepare(
        base + ".Corrected.HVG.Varnorm.h5ad", components=[a.k], n_iter=a.n_iter, seed=14,
        tpm_fn=base + ".TP10K.h5ad", genes_file=base + ".Corrected.HVGs.txt"))
    t["prepare"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    staged("factorize", lambda: obj.factorize(verbose=False))
    t["factorize"] = time.perf_counter() - t0
    t0 = time.perf_counter()

    def cc():
        obj.combine()
        obj.consensus(a.k, density_threshold=2.0, show_clustering=False)

    staged("combine_consensus", cc)
    t["combine_consensus"] = time.perf_counter() - t0
    print(json.dumps({
        "metric": "Harmony + cNMF end-to-end wall-clock", "unit": "s",
        "value": round(sum(v for k, v in t.items() if k != "simulate"), 2),
        "stages_s": {k: round(v, 2) for k, v in t.items()},
        "gpu_busy_s": busy or None,
        "harmony": getattr(p, "harmony_info_", None),
        "config": {"cells": a.cells, "genes": a.genes, "hvg": a.hvg, "covariates": 4,
                   "k": a.k, "n_iter": a.n_iter, "max_iter_harmony": a.max_iter_harmony,
                   "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu"},
        "data": "synthetic sparse counts, planted programs x 4 multiplicative covariate effects"}))


if __name__ == "__main__":
    main()

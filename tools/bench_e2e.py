"""End-to-end wall-clock of the whole cNMF pipeline (BASELINE.json config 2:
"PBMC-scale 10k cells x 2k HVGs, K=5..13, n_iter=100 on 1 MI355X").

    python tools/bench_e2e.py [--cells 10000 --genes 8000 --hvg 2000 --kmin 5 --kmax 13 --n-iter 100]

Synthetic sparse counts (planted programs, utils/synthetic.py) written as .h5ad; then
prepare -> factorize -> combine -> k_selection_plot -> consensus at the middle K, each
stage timed.  Prints one JSON line (stage seconds, total, replicates/s of factorize).
The reference's own figure for its tutorial-scale run (120 replicates, 2.7k cells) is
"roughly 4 minutes" on CPU.
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pandas as pd  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd import cNMF  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402
from cnmf_torch_amd.utils.h5ad import write_h5ad  # noqa: E402
from cnmf_torch_amd.utils.plotting import flush_figures  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402


def _profile_kstats(obj, kmid, a, warm: bool) -> None:
    """cProfile one K's k-selection statistics (consensus up to its stats), serially."""
    import cProfile
    import pstats

    def kstats():
        obj.consensus(kmid, skip_density_and_return_after_stats=True, show_clustering=False,
                      close_clustergram_fig=True, kmeans_backend=a.kmeans_backend)
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    if warm:
        kstats()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    kstats()
    pr.disable()
    with open(a.profile_kstats, "w") as fh:
        fh.write(f"==== k-selection statistics of K={kmid}, serial, "
                 f"{'warm' if warm else 'first call'}: {time.perf_counter() - t0:.3f} s ====\n")
        pstats.Stats(pr, stream=fh).sort_stats("cumulative").print_stats(45)
        pstats.Stats(pr, stream=fh).sort_stats("tottime").print_stats(25)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--genes", type=int, default=8000)
    ap.add_argument("--hvg", type=int, default=2000)
    ap.add_argument("--programs", type=int, default=9)
    ap.add_argument("--kmin", type=int, default=5)
    ap.add_argument("--kmax", type=int, default=13)
    ap.add_argument("--n-iter", type=int, default=100)
    ap.add_argument("--threshold", type=float, default=0.1)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--profile", default=None, help="cProfile every stage into this file")
    ap.add_argument("--kmeans-backend", default="auto", choices=["auto", "sklearn", "device"],
                    help="sklearn = the reference's exact KMeans; device = batched GPU restarts")
    ap.add_argument("--profile-kstats", default=None,
                    help="after the pipeline: cProfile ONE K's k-selection statistics "
                         "(consensus up to its stats, serial, warm) into this file -- the "
                         "stage itself runs them on worker threads cProfile does not see")
    ap.add_argument("--kstats-cold", action="store_true",
                    help="with --profile-kstats: profile the FIRST call instead (right after "
                         "combine, before the k-selection stage): the first-use costs")
    a = ap.parse_args()
    work = a.workdir or tempfile.mkdtemp(prefix="cnmf_e2e_")
    X, cells, genes = simulate_counts(a.cells, a.genes, a.programs, seed=0, sparse=True)
    counts = os.path.join(work, "counts.h5ad")
    write_h5ad(counts, AnnData(X=X, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
    ks = list(range(a.kmin, a.kmax + 1))
    t = {}
    obj = cNMF(output_dir=work, name="e2e")
    kmid = ks[len(ks) // 2]
    stages = [("prepare", lambda: obj.prepare(counts, components=ks, n_iter=a.n_iter, seed=14,
                                              num_highvar_genes=a.hvg)),
              ("factorize", lambda: obj.factorize(verbose=False)),
              ("combine", obj.combine),
              ("k_selection_plot", lambda: obj.k_selection_plot(close_fig=True,
                                                               kmeans_backend=a.kmeans_backend,
                                                               wait_figures=False)),
              ("consensus", lambda: obj.consensus(kmid, density_threshold=a.threshold,
                                                  show_clustering=True,
                                                  close_clustergram_fig=True,
                                                  kmeans_backend=a.kmeans_backend,
                                                  wait_figures=False)),
              # the figures render while later stages compute (as the CLI does); the
              # pipeline is done once the last PNG is on disk
              ("figures", flush_figures)]
    prof_out = open(a.profile, "w") if a.profile else None
    if a.profile_kstats and a.kstats_cold:      # prepare .. combine, then the cold probe
        for name, fn in stages[:3]:
            t0 = time.perf_counter()
            fn()
            t[name] = time.perf_counter() - t0
        stages = stages[3:]
        _profile_kstats(obj, kmid, a, warm=False)
    for name, fn in stages:
        if prof_out:
            import cProfile
            import pstats

            pr = cProfile.Profile()
            pr.enable()
        t0 = time.perf_counter()
        fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t[name] = time.perf_counter() - t0
        if prof_out:
            pr.disable()
            prof_out.write(f"==== {name} ====\n")
            pstats.Stats(pr, stream=prof_out).sort_stats("cumulative").print_stats(30)
    if prof_out:
        prof_out.close()
    if a.profile_kstats and not a.kstats_cold:
        _profile_kstats(obj, kmid, a, warm=True)
    total = sum(t.values())
    n_rep = len(ks) * a.n_iter
    print(json.dumps({
        "metric": "cNMF end-to-end wall-clock", "unit": "s", "value": round(total, 3),
        "stages_s": {k: round(v, 3) for k, v in t.items()},
        "factorize_replicates_per_s": round(n_rep / t["factorize"], 2),
        # factorize = its solves + the wait for the 900 replicate files (filesystem-bound)
        "factorize_split_s": {k: round(v, 4) for k, v in
                              getattr(obj, "factorize_stats", {}).items()},
        "config": {"kmeans_backend": a.kmeans_backend, "cells": a.cells, "genes": a.genes, "hvg": a.hvg, "k": [a.kmin, a.kmax],
                   "n_iter": a.n_iter, "replicates": n_rep,
                   "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu"},
        "data": "synthetic sparse counts (planted programs)"}))


if __name__ == "__main__":
    main()

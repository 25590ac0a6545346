"""End-to-end cNMF on a simulated data set (the reference's simulated-data tutorial,
Tutorials/analyze_simulated_example_data.ipynb, as a script).

    python examples/simulated_end_to_end.py --out /tmp/cnmf_demo [--cells 3000 --genes 1500]

Simulates Poisson counts from planted gene-expression programs, runs the five cNMF
stages through the Python API (on the GPU when one is visible), and reports how well the
consensus spectra recover the planted programs.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pandas as pd  # noqa: E402

from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="./cnmf_demo")
    ap.add_argument("--cells", type=int, default=2000)
    ap.add_argument("--genes", type=int, default=1000)
    ap.add_argument("--programs", type=int, default=6)
    ap.add_argument("--n-iter", type=int, default=20)
    ap.add_argument("--threshold", type=float, default=0.1)
    a = ap.parse_args()

    X, cells, genes = simulate_counts(a.cells, a.genes, a.programs, seed=0, sparse=False)
    os.makedirs(a.out, exist_ok=True)
    counts_fn = os.path.join(a.out, "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), counts_fn)

    t0 = time.perf_counter()
    obj = cNMF(output_dir=a.out, name="sim")
    ks = list(range(a.programs - 2, a.programs + 3))
    obj.prepare(counts_fn, components=ks, n_iter=a.n_iter, seed=14,
                num_highvar_genes=min(1500, a.genes))
    t1 = time.perf_counter()
    obj.factorize()
    t2 = time.perf_counter()
    obj.combine()
    obj.k_selection_plot(close_fig=True)
    obj.consensus(a.programs, density_threshold=a.threshold, show_clustering=True,
                  close_clustergram_fig=True)
    t3 = time.perf_counter()
    usage, scores, tpm, top = obj.load_results(K=a.programs, density_threshold=a.threshold)
    print(f"prepare {t1 - t0:.1f}s  factorize {t2 - t1:.1f}s "
          f"({len(ks) * a.n_iter / (t2 - t1):.1f} replicates/s)  combine+consensus {t3 - t2:.1f}s")
    print("k-selection stats:")
    print(load_df_from_npz(obj.paths["k_selection_stats"]))
    print("top genes per program:")
    print(top.head(5).to_string())


if __name__ == "__main__":
    main()

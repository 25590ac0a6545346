"""Harmony batch correction + cNMF (the reference's BaronEtAl batch-correction tutorial,
Tutorials/analyze_batcheffectcorrect_BaronEtAl.ipynb, on simulated data).

    python examples/batch_correction.py --out /tmp/cnmf_bc

Adds a multiplicative per-batch gene effect to simulated counts, runs
Preprocess.preprocess_for_cnmf(harmony_vars='batch') (Harmony's R-update runs as fused HIP
kernels on the GPU), and factorizes the corrected matrix with the corrected TP10K as TPM.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import scipy.sparse as sp  # noqa: E402

from cnmf_torch_amd import Preprocess, cNMF  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402
from cnmf_torch_amd.utils.h5ad import write_h5ad  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="./cnmf_bc")
    ap.add_argument("--cells", type=int, default=3000)
    ap.add_argument("--genes", type=int, default=1500)
    ap.add_argument("--batches", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    rs = np.random.default_rng(0)
    X, cells, genes = simulate_counts(a.cells, a.genes, 5, seed=1, sparse=False)
    batch = rs.integers(0, a.batches, a.cells)
    effect = rs.lognormal(0.0, 0.5, (a.batches, a.genes))
    X = rs.poisson(X * effect[batch]).astype(np.float32)
    obs = pd.DataFrame({"batch": pd.Categorical([f"b{b}" for b in batch])}, index=cells)
    adata = AnnData(X=sp.csr_matrix(X), obs=obs, var=pd.DataFrame(index=genes))

    p = Preprocess(random_seed=0)
    adata = p.filter_adata(adata, min_cells_per_gene=10, min_counts_per_cell=50, makeplots=False)
    base = os.path.join(a.out, "bc")
    corrected, tp10k, hvgs = p.preprocess_for_cnmf(adata, harmony_vars="batch",
                                                   n_top_rna_genes=1000, makeplots=False,
                                                   save_output_base=base)
    obj = cNMF(output_dir=a.out, name="bc_cnmf")
    obj.prepare(base + ".Corrected.HVG.Varnorm.h5ad", components=[4, 5, 6], n_iter=10,
                seed=14, tpm_fn=base + ".TP10K.h5ad", genes_file=base + ".Corrected.HVGs.txt")
    obj.factorize()
    obj.combine()
    obj.consensus(5, density_threshold=0.2, show_clustering=False)
    usage, scores, tpm, top = obj.load_results(K=5, density_threshold=0.2)
    print(usage.groupby(obs.loc[usage.index, "batch"].astype(str).values).mean().round(3))


if __name__ == "__main__":
    main()

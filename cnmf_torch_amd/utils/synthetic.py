"""Synthetic single-cell count matrices with planted gene expression programs.

A light stand-in for the scsim simulator the reference's tutorials use
(Extras/simulate_example_data.ipynb:114: K programs, identity + activity programs,
per-cell library sizes).  There is no network here, so benchmarks and tests use these
matrices: planted usages U (cells x K, Dirichlet, a few activity programs spread over
cell types), planted spectra S (K x genes, sparse log-normal), library sizes
log-normal, counts ~ Poisson(lib * (U S)_normalised).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import scipy.sparse as sp


def simulate_counts(n_cells: int = 1000, n_genes: int = 500, n_programs: int = 5,
                    seed: int = 0, mean_lib: float = 2000.0, sparse: bool = True,
                    program_frac: float = 0.15, dirichlet_alpha: float = 0.3,
                    return_truth: bool = False):
    rs = np.random.default_rng(seed)
    K = n_programs
    # spectra: each program up-regulates a random subset of genes
    base = rs.lognormal(mean=0.0, sigma=1.0, size=n_genes)
    S = np.tile(base, (K, 1))
    for k in range(K):
        genes = rs.choice(n_genes, size=max(1, int(program_frac * n_genes)), replace=False)
        S[k, genes] *= rs.lognormal(mean=1.5, sigma=0.5, size=genes.size)
    S /= S.sum(axis=1, keepdims=True)
    U = rs.dirichlet(np.full(K, dirichlet_alpha), size=n_cells)
    lib = rs.lognormal(mean=np.log(mean_lib), sigma=0.35, size=n_cells)
    lam = (U @ S) * lib[:, None]
    counts = rs.poisson(lam).astype(np.float32)
    # make sure no cell / gene is entirely empty (cNMF prepare rejects zero-count cells)
    empty = counts.sum(axis=1) == 0
    if empty.any():
        counts[empty, rs.integers(0, n_genes, empty.sum())] = 1.0
    X = sp.csr_matrix(counts) if sparse else counts
    cells = [f"cell{i}" for i in range(n_cells)]
    genes = [f"gene{i}" for i in range(n_genes)]
    if return_truth:
        return X, cells, genes, U, S
    return X, cells, genes


def simulate_counts_df(n_cells=1000, n_genes=500, n_programs=5, seed=0, **kw) -> pd.DataFrame:
    X, cells, genes = simulate_counts(n_cells, n_genes, n_programs, seed, sparse=False, **kw)
    return pd.DataFrame(X, index=cells, columns=genes)


def normalized_counts_matrix(n_cells: int, n_genes: int, n_programs: int = 10, seed: int = 0,
                             dtype=np.float32) -> np.ndarray:
    """Dense matrix shaped like cNMF's ``norm_counts`` (HVG subset of raw counts scaled
    to unit variance per gene, cnmf.py:670-681): what ``factorize`` consumes."""
    X, _, _ = simulate_counts(n_cells, n_genes, n_programs, seed, sparse=False)
    sd = X.std(axis=0, ddof=1)
    sd[sd == 0] = 1.0
    return (X / sd).astype(dtype)

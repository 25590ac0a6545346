"""Gene statistics, over-dispersed gene selection and TPM (C6-C9; cnmf.py:128-247).

Semantics follow the reference exactly: column mean / variance with ddof=0
(``StandardScaler(with_mean=False)``, cnmf.py:128-131), the Fano-factor model with
A = min CV of the 20 highest-mean genes and B^2 = median Fano inside the 10-90 %
winsor box (cnmf.py:143-156), selection of the top ``numgenes`` by Fano ratio or, with
``numgenes=None``, by threshold ``T = 1 + std(winsorised Fano)`` and mean > 0.5
(cnmf.py:160-171).  The per-gene vectors are small, so ranking uses pandas for
identical tie-breaking; the column statistics over the (cells x genes) matrix run on
the GPU for device tensors (one pass, float64 accumulation).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import scipy.sparse as sp
import torch


def sparse_mean_var(X):
    """Column mean and ddof=0 variance of a scipy sparse matrix: sklearn's corrected
    two-pass CSR algorithm (``sklearn.utils.sparsefuncs.mean_variance_axis``, which
    ``StandardScaler(with_mean=False).fit`` runs, cnmf.py:128-131) re-expressed as
    float64 bincounts that accumulate in the same (row-major data) order -- without
    importing sklearn, whose import alone was ~1 s of every ``prepare``."""
    X = sp.csr_matrix(X)
    N, G = X.shape
    from ..utils.io import _npzio
    if _npzio is not None and X.dtype in (np.float32, np.float64):
        mean, var = _npzio.csr_mean_var(X.data, X.indices, N, G)   # native, same bits
        if X.dtype == np.float32:
            return mean.astype(np.float32).astype(np.float64), var.astype(np.float32).astype(np.float64)
        return mean, var
    data = np.asarray(X.data, dtype=np.float64)
    idx = X.indices
    nnz = np.bincount(idx, minlength=G)
    mean = np.bincount(idx, weights=data, minlength=G) / float(N)
    diff = data - mean[idx]
    corr = np.bincount(idx, weights=diff, minlength=G)
    var = np.bincount(idx, weights=diff * diff, minlength=G)
    miss = (N - nnz).astype(np.float64)
    has = nnz != N
    corr = np.where(has, corr - miss * mean, corr)
    corr = corr ** 2 / float(N)
    var = np.where(has, var + miss * mean ** 2, var)
    var = (var - corr) / float(N)
    if X.dtype == np.float32:     # sklearn's float32 specialisation returns float32 values
        return mean.astype(np.float32).astype(np.float64), var.astype(np.float32).astype(np.float64)
    return mean, var


def get_mean_var(X):
    """Column mean and ddof=0 variance of a dense/sparse/torch matrix or a device CSR
    (cnmf.py:128-131)."""
    from ..ops import sparse as sops

    if isinstance(X, sops.DeviceCSR):
        mean, var = sops.mean_var(X, ddof=0)
        return mean.cpu().numpy(), var.cpu().numpy()
    if isinstance(X, torch.Tensor):
        Xd = X.to(torch.float64)
        mean = Xd.mean(dim=0)
        var = (Xd * Xd).mean(dim=0) - mean * mean
        return mean.cpu().numpy(), torch.clamp(var, min=0).cpu().numpy()
    if sp.issparse(X):
        return sparse_mean_var(X)
    from sklearn.preprocessing import StandardScaler

    sc = StandardScaler(with_mean=False)
    sc.fit(X)
    return sc.mean_, sc.var_


def _fano_model(gene_mean: pd.Series, gene_var: pd.Series, expected_fano_threshold=None,
                minimal_mean: float = 0.5, numgenes=None):
    gene_fano = gene_var / gene_mean
    # expected Fano line: A^2 * mean + B^2
    top_by_mean = gene_mean.sort_values(ascending=False)[:20].index
    A = (np.sqrt(gene_var) / gene_mean)[top_by_mean].min()
    m_lo, m_hi = gene_mean.quantile([0.10, 0.90])
    f_lo, f_hi = gene_fano.quantile([0.10, 0.90])
    box = (gene_fano > f_lo) & (gene_fano < f_hi) & (gene_mean > m_lo) & (gene_mean < m_hi)
    B = np.sqrt(gene_fano[box].median())
    expected = (A ** 2) * gene_mean + B ** 2
    ratio = gene_fano / expected
    if numgenes is not None:
        chosen = ratio.sort_values(ascending=False).index[:numgenes]
        high_var = ratio.index.isin(chosen)
        T = None
    else:
        T = (1.0 + gene_fano[box].std()) if not expected_fano_threshold else expected_fano_threshold
        high_var = (ratio > T) & (gene_mean > minimal_mean)
    stats = pd.DataFrame({"mean": gene_mean, "var": gene_var, "fano": gene_fano,
                          "expected_fano": expected, "high_var": high_var, "fano_ratio": ratio})
    params = {"A": A, "B": B, "T": T, "minimal_mean": minimal_mean}
    return stats, params


def get_highvar_genes_sparse(expression, expected_fano_threshold=None, minimal_mean=0.5,
                             numgenes=None):
    """Over-dispersed genes of a sparse (or torch) matrix (cnmf.py:133-184)."""
    mean, var = get_mean_var(expression)
    return _fano_model(pd.Series(mean), pd.Series(var), expected_fano_threshold, minimal_mean,
                       numgenes)


def get_highvar_genes(input_counts, expected_fano_threshold=None, minimal_mean=0.5, numgenes=None):
    """Dense variant (cnmf.py:188-238): numpy mean / var(ddof=0)."""
    X = np.asarray(input_counts)
    mean = pd.Series(X.mean(axis=0).astype(float))
    var = pd.Series(X.var(ddof=0, axis=0).astype(float))
    return _fano_model(mean, var, expected_fano_threshold, minimal_mean, numgenes)


def compute_tpm(input_counts):
    """Per-cell scaling to 1e6 total (``sc.pp.normalize_total(target_sum=1e6)``, cnmf.py:241-247)."""
    from .pp import normalize_total

    return normalize_total(input_counts, target_sum=1e6, copy=True)

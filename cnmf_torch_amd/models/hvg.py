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

import math

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


def _digits_to_ints(d: np.ndarray) -> list:
    """Per-row Python ints of base-2^32 signed int64 digit vectors (carries propagated in
    numpy, then one int.from_bytes per row)."""
    d = np.array(d, dtype=np.int64, copy=True)
    D = d.shape[1]
    for i in range(D - 1):            # arithmetic shift: floor division by 2^32
        carry = d[:, i] >> 32
        d[:, i] -= carry << 32
        d[:, i + 1] += carry
    top = d[:, D - 1]
    low = d[:, :D - 1].astype("<u4")  # every lower digit now in [0, 2^32)
    out = []
    for j in range(d.shape[0]):
        v = int.from_bytes(low[j].tobytes(), "little") + (int(top[j]) << (32 * (D - 1)))
        out.append(v)
    return out


DEVICE_MOMENT_BLOCKS = 0      # row blocks whose digits ran on the GPU (tests, tracing)


def _device_moment_digits(X, device, block_bytes: int = 2 << 30):
    """exact_moment_digits of a HOST scipy-sparse / numpy matrix on the GPU: row blocks
    of at most ``block_bytes`` dense bytes go to the device (CSR blocks are densified
    there), exact_moments.hip adds each block's digits into one int64 accumulator --
    integer sums, so the digits are the host path's bit for bit."""
    global DEVICE_MOMENT_BLOCKS
    from .. import ops

    N, G = X.shape
    dt = torch.float64 if X.dtype == np.float64 else torch.float32
    esz = 8 if dt == torch.float64 else 4
    rows = max(1, min(N, block_bytes // max(1, G * esz)))
    acc = torch.zeros((G, ops.EXACT_D1 + ops.EXACT_D2), dtype=torch.int64, device=device)
    bad = torch.zeros(1, dtype=torch.int64, device=device)
    Xc = sp.csr_matrix(X) if sp.issparse(X) else None
    for a in range(0, N, rows):
        b = min(N, a + rows)
        if Xc is not None:
            blk = Xc[a:b]
            dense = torch.zeros((b - a, G), dtype=dt, device=device)
            if blk.nnz:
                r = np.repeat(np.arange(b - a, dtype=np.int64), np.diff(blk.indptr))
                idx = torch.from_numpy(r * G + blk.indices.astype(np.int64)).to(device)
                dense.view(-1).index_copy_(0, idx, torch.from_numpy(
                    np.asarray(blk.data, dtype=np.float64 if esz == 8 else np.float32)).to(device))
        else:
            dense = torch.from_numpy(np.ascontiguousarray(
                X[a:b], dtype=np.float64 if esz == 8 else np.float32)).to(device)
        ops.exact_moments(dense, acc=acc, bad_acc=bad)
        DEVICE_MOMENT_BLOCKS += 1
        del dense
    o = acc.cpu().numpy()
    return o[:, :ops.EXACT_D1].copy(), o[:, ops.EXACT_D1:].copy(), int(bad.item())


def exact_moment_digits(X, threads: int = 16, device=None):
    """Exact per-column (sum x, sum x^2) of a scipy sparse / numpy dense / torch matrix as
    integer digit arrays ((G, D1), (G, D2) int64) plus the number of values outside the
    exact window (|x| in [2^-126, 2^127]), or None without the native module.  Integer
    digits add exactly: the sums of any row partition (threads, ranks) are the same
    integers, so statistics built from them do not depend on how the cells are split.
    ``device`` (a GPU): a host matrix's digits are formed there, block by block
    (_device_moment_digits) -- the same integers."""
    from ..utils.io import _npzio
    if device is not None and torch.device(device).type == "cuda" and \
            not isinstance(X, torch.Tensor) and X.dtype in (np.float32, np.float64):
        from .. import ops
        if ops.native_available() and X.shape[1] > 0:
            return _device_moment_digits(X, torch.device(device))
    if _npzio is None or not hasattr(_npzio, "exact_col_moments"):
        return None
    if isinstance(X, torch.Tensor):
        if X.is_cuda:
            from .. import ops
            if ops.use_native(X):
                return ops.exact_moments(X)
            # torch-ops debug mode (CNMF_FORCE_TORCH_OPS / eager_ops): the host digits of
            # the same values -- the same integers the kernel sums
            X = X.cpu()
        X = X.numpy()
    if sp.issparse(X):
        Xc = sp.csr_matrix(X)
        data = Xc.data if Xc.data.dtype in (np.float32, np.float64) else Xc.data.astype(np.float64)
        return _npzio.exact_col_moments(data, Xc.indices, int(Xc.shape[1]), threads)
    A = np.asarray(X)
    if A.dtype not in (np.float32, np.float64):
        A = A.astype(np.float64)
    return _npzio.exact_col_moments(np.ascontiguousarray(A), None, int(A.shape[1]), threads)


def exact_mean_var_from_digits(d1, d2, n: int, ddof: int = 0):
    """Column mean and variance (ddof) from exact moment digits: mean = S1 / n and
    var = (n S2 - S1^2) / (n (n - ddof)), each computed in integers and rounded ONCE to
    float64 (numpy/sklearn's two-pass float64 sums round at every add)."""
    from ..utils.io import _npzio
    lsb1, lsb2 = int(_npzio.EXACT_LSB1), int(_npzio.EXACT_LSB2)
    s1 = _digits_to_ints(d1)
    s2 = _digits_to_ints(d2)
    n = int(n)
    G = len(s1)
    mean = np.empty(G)
    var = np.empty(G)
    den = n * (n - ddof) if n > ddof else 0
    for j in range(G):
        mean[j] = math.ldexp(s1[j] / n, lsb1) if n else 0.0
        if den:
            num = n * s2[j] - s1[j] * s1[j]       # in units of 2^lsb2 (= 2^(2 lsb1))
            var[j] = math.ldexp(num / den, lsb2) if num > 0 else 0.0
        else:
            var[j] = float("nan")
    return mean, var


def exact_mean_var(X, ddof: int = 0, comm=None, device=None):
    """Exact column mean / variance (see exact_mean_var_from_digits) of a row block X; with
    ``comm`` the digits are all-reduced first (integer sums: the sharded statistics equal
    the single-process ones bit for bit).  None when the exact path is unavailable or a
    value lies outside its window on any rank (callers then use floating point).
    ``device``: form a host X's digits on that GPU (exact_moment_digits)."""
    got = exact_moment_digits(X, device=device)
    n_loc = int(X.shape[0])
    flag = 1 if got is None else (1 if int(got[2]) else 0)
    if comm is not None and comm.is_distributed:
        flag = comm.allreduce_max_int(flag)
    if flag:
        return None
    d1, d2 = torch.from_numpy(np.ascontiguousarray(got[0])), torch.from_numpy(np.ascontiguousarray(got[1]))
    n = n_loc
    if comm is not None and comm.is_distributed:
        flat = torch.cat([d1.reshape(-1), d2.reshape(-1)])
        comm.allreduce_(flat)
        d1 = flat[:d1.numel()].view_as(d1)
        d2 = flat[d1.numel():].view_as(d2)
        n = int(round(comm.allreduce_scalar(float(n_loc))))
    return exact_mean_var_from_digits(d1.numpy(), d2.numpy(), n, ddof)


def get_mean_var(X):
    """Column mean and ddof=0 variance of a dense/sparse/torch matrix or a device CSR
    (cnmf.py:128-131).  Host and dense-device matrices take the exact path
    (exact_mean_var: the moments summed in integers, rounded once), so the statistics do
    not depend on the device or on a row sharding; float32 input keeps sklearn's float32
    results."""
    from ..ops import sparse as sops

    if not isinstance(X, sops.DeviceCSR):
        ex = exact_mean_var(X, 0)
        if ex is not None:
            mean, var = ex
            if getattr(X, "dtype", None) in (np.float32, torch.float32):
                return mean.astype(np.float32).astype(np.float64), \
                    var.astype(np.float32).astype(np.float64)
            return mean, var
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
    ex = exact_mean_var(X, 0)
    if ex is not None:
        mean, var = (pd.Series(v) for v in ex)
    else:
        mean = pd.Series(X.mean(axis=0).astype(float))
        var = pd.Series(X.var(ddof=0, axis=0).astype(float))
    return _fano_model(mean, var, expected_fano_threshold, minimal_mean, numgenes)


def compute_tpm(input_counts):
    """Per-cell scaling to 1e6 total (``sc.pp.normalize_total(target_sum=1e6)``, cnmf.py:241-247)."""
    from .pp import normalize_total

    return normalize_total(input_counts, target_sum=1e6, copy=True)

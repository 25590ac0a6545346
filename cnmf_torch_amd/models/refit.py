"""Usage / spectra refit with the other factor fixed (C10, cnmf.py:260-388).

``fit_H_online`` reproduces the reference's online MU refit: numerator ``x W^T`` per
row chunk, ``W W^T`` precomputed, up to ``chunk_max_iter`` MU steps per chunk with the
chunk-level stop ``||h_new - h|| / (||h|| + eps) < h_tol`` and ``rates = 0`` where the
denominator < eps (cnmf.py:348-381).  Differences by design:

* X is never densified as a whole: the numerator ``W X^T`` is streamed over row blocks
  (dense, CSR, numpy or torch input) straight into device memory; after that X is not
  needed again -- every MU step only touches the (K x n) numerator and H.
* the random init is seeded (Philox stream 2, ``random_state``) instead of the
  unseeded ``torch.rand`` of cnmf.py:343, so consensus is reproducible.
* all chunks run in ONE launch of the fused solve kernel (one workgroup per chunk,
  on-device convergence), instead of a host-synchronised loop per chunk.

``fit_spectra_online`` is ``refit_spectra`` (cnmf.py:979-994, ``refit_usage(X.T,
usage.T).T``) without materialising ``X.T`` densely: its numerator is ``U^T X``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import scipy.sparse as sp
import torch

from .. import ops
from ..ops import sparse as sops
from ..utils import rng


def _to_numpy_2d(a):
    if isinstance(a, pd.DataFrame):
        return a.values
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return a


def _block_to_device(blk, device, dtype):
    if sp.issparse(blk):
        blk = blk.toarray()
    if isinstance(blk, torch.Tensor):
        return blk.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(blk), dtype=dtype).to(device)


def numer_rows(W: torch.Tensor, X, block: int = 16384) -> torch.Tensor:
    """W (K x G, device) times X^T for X (n x G) in any format -> (K x n) on W's device.
    A device CSR (ops.sparse.DeviceCSR, possibly a scaled/subset view) goes through the
    CSR SpMM kernel; nothing is densified."""
    if isinstance(X, sops.DeviceCSR):
        return sops.spmm(X, W.t()).t().contiguous().to(W.dtype)
    n = X.shape[0]
    out = torch.empty((W.shape[0], n), device=W.device, dtype=W.dtype)
    if isinstance(X, torch.Tensor) and X.device == W.device:
        torch.mm(W, X.to(W.dtype).t(), out=out)
        return out
    for a in range(0, n, block):
        b = min(n, a + block)
        xb = _block_to_device(X[a:b], W.device, W.dtype)
        torch.mm(W, xb.t(), out=out[:, a:b])
    return out


def numer_cols(U: torch.Tensor, X, block: int = 16384) -> torch.Tensor:
    """U^T X for U (n x K, device) and X (n x G) in any format -> (K x G).  A device CSR
    goes through the deterministic transposed-SpMM kernel (float64 accumulation)."""
    if isinstance(X, sops.DeviceCSR):
        return sops.tspmm(X, U).t().to(U.dtype).contiguous()
    n, G = X.shape
    out = torch.zeros((U.shape[1], G), device=U.device, dtype=U.dtype)
    if isinstance(X, torch.Tensor) and X.device == U.device:
        return torch.mm(U.t(), X.to(U.dtype))
    for a in range(0, n, block):
        b = min(n, a + block)
        xb = _block_to_device(X[a:b], U.device, U.dtype)
        out += U[a:b].t() @ xb
    return out


def chunked_solve(HT: torch.Tensor, numerT: torch.Tensor, gram: torch.Tensor, chunk_size: int,
                  chunk_max_iter: int, h_tol: float, l1_num: float = 0.0, l2: float = 0.0,
                  eps: float = 1e-16, algo: str = "mu") -> torch.Tensor:
    """Independent per-chunk solves of HT (K x n) in place; one launch for all full chunks.
    On the GPU a rank without its own kernel instantiation (K > 32 not a multiple of 8,
    64 < K <= 128 not a multiple of 16) is solved padded with zero components, which stay zero
    and leave the Gram products and the objective unchanged (models.nmf.native_rank)."""
    K, n = HT.shape
    if HT.device.type == "cuda" and algo != "bpp" and ops.use_native(HT):
        from .nmf import _warn_once, kernel_max_rank, native_rank

        kmax = kernel_max_rank(2.0, algo)
        if kmax is not None and K > kmax:    # no kernel for this rank: the PyTorch ops on the same GPU, logged
            _warn_once(f"refit K={K}: the native gfx950 solve covers K <= {kmax}; this "
                       "refit runs the eager PyTorch ops on the GPU (slower)")
            with ops.eager_ops():
                return chunked_solve(HT, numerT, gram, chunk_size, chunk_max_iter, h_tol,
                                     l1_num=l1_num, l2=l2, eps=eps, algo=algo)

        Kp = native_rank(K)
        if Kp != K:
            HTp = torch.zeros((Kp, n), device=HT.device, dtype=HT.dtype)
            Np = torch.zeros((Kp, n), device=HT.device, dtype=numerT.dtype)
            Gp = torch.zeros((Kp, Kp), device=HT.device, dtype=gram.dtype)
            HTp[:K], Np[:K], Gp[:K, :K] = HT, numerT, gram
            chunked_solve(HTp, Np, Gp, chunk_size, chunk_max_iter, h_tol, l1_num=l1_num,
                          l2=l2, eps=eps, algo=algo)
            HT.copy_(HTp[:K])
            return HT
    c = max(1, min(int(chunk_size), n))
    full = n // c
    g1 = gram.reshape(1, K, K).contiguous()
    if full:
        xv = HT.as_strided((full, K, c), (c, HT.stride(0), 1), HT.storage_offset())
        nv = numerT.as_strided((full, K, c), (c, numerT.stride(0), 1), numerT.storage_offset())
        ops.solve(algo, xv, nv, g1.expand(full, K, K).contiguous(), max_iter=chunk_max_iter,
                  tol=h_tol, l1_num=l1_num, l2=l2, eps=eps)
    if full * c < n:
        a = full * c
        ops.solve(algo, HT[:, a:].unsqueeze(0), numerT[:, a:].unsqueeze(0), g1,
                  max_iter=chunk_max_iter, tol=h_tol, l1_num=l1_num, l2=l2, eps=eps)
    if HT.device.type == "cuda":
        # few chunks take the cooperative path: a solve whose workgroups could not all be
        # resident gave up waiting -> its usages are wrong; fail here, not downstream
        ops.coop_check(HT.device)
    return HT


def _init_HT(K: int, n: int, H_init, device, dtype, random_state: int,
             row_offset: int = 0) -> torch.Tensor:
    if H_init is not None:
        H0 = torch.as_tensor(np.asarray(_to_numpy_2d(H_init)), dtype=dtype)
        return torch.clamp(H0, min=0.0).t().contiguous().to(device)
    HT = torch.empty((K, n), device=device, dtype=dtype)
    if n:
        ops.philox_fill(HT.as_strided((1, n, K), (K * n, 1, n)),
                        torch.tensor([int(random_state)]), torch.tensor([1.0]), rng.STREAM_REFIT,
                        mode=1, row_offset=int(row_offset))
    return HT


def col_block(X, g0: int, g1: int):
    """Columns [g0, g1) of X (dense numpy/torch, scipy sparse or a plain DeviceCSR, the
    latter as a lazy column-map view) -- a rank's gene block under gene-axis sharding."""
    if isinstance(X, sops.DeviceCSR):
        if X.xf:
            raise ValueError("col_block: transformed DeviceCSR views are not sharded")
        cmap = np.full(X.shape[1], -1, np.int32)
        cmap[g0:g1] = np.arange(g1 - g0, dtype=np.int32)
        return X.view(col_map=cmap, n_out=g1 - g0)
    if isinstance(X, pd.DataFrame):
        return X.iloc[:, g0:g1]
    return X[:, g0:g1]


def gene_blocks(G: int, chunk: int, world: int) -> list[tuple[int, int]]:
    """Gene-axis shards made of WHOLE refit chunks (the chunked solve's convergence is
    decided per chunk), so a sharded spectra refit equals the unsharded one."""
    c = max(1, int(chunk))
    n_chunks = -(-G // c) if G else 0
    out = []
    for r in range(world):
        a = (n_chunks * r // world) * c
        b = min(G, (n_chunks * (r + 1) // world) * c)
        out.append((min(a, G), b))
    return out


def fit_H_online(X, W, H_init=None, chunk_size: int = 5000, chunk_max_iter: int = 200,
                 h_tol: float = 0.05, l1_reg_H: float = 0.0, l2_reg_H: float = 0.0,
                 epsilon: float = 1e-16, device="cpu", random_state: int = 0,
                 return_tensor: bool = False):
    """Refit H (n x K) >= 0 minimising ||X - H W|| with W (K x G) fixed (cnmf.py:260)."""
    dev = torch.device(device)
    dtype = torch.float32
    Wt = torch.as_tensor(np.asarray(_to_numpy_2d(W), dtype=np.float32)).to(dev)
    Xv = X.values if isinstance(X, pd.DataFrame) else X
    K = Wt.shape[0]
    n = Xv.shape[0]
    numerT = numer_rows(Wt, Xv)
    gram = ops.small_gram(Wt, rows_are_points=False)      # W W^T (segsum.hip)
    HT = _init_HT(K, n, H_init, dev, dtype, random_state)
    chunked_solve(HT, numerT, gram, chunk_size, chunk_max_iter, h_tol, l1_num=l1_reg_H,
                  l2=l2_reg_H, eps=epsilon)
    if return_tensor:
        return HT.t()
    return HT.t().cpu().numpy()


def fit_spectra_online(X, usage, chunk_size: int = 5000, chunk_max_iter: int = 200,
                       h_tol: float = 0.05, l1_reg: float = 0.0, epsilon: float = 1e-16,
                       device="cpu", random_state: int = 0, col_offset: int = 0):
    """Refit spectra S (K x G) >= 0 minimising ||X - U S|| with usages U (n x K) fixed.

    Equals ``fit_H_online(X.T, U.T).T`` (cnmf.py:994): chunks run over genes.
    ``col_offset``: X holds the genes [col_offset, col_offset + G) of a larger matrix (a
    gene-sharded rank): the seeded init is taken at those genes, so shards reproduce
    the unsharded refit when they hold whole chunks (gene_blocks)."""
    dev = torch.device(device)
    Ut = torch.as_tensor(np.asarray(_to_numpy_2d(usage), dtype=np.float32)).to(dev)
    Xv = X.values if isinstance(X, pd.DataFrame) else X
    K = Ut.shape[1]
    G = Xv.shape[1]
    numerT = numer_cols(Ut, Xv)          # (K x G) = (X^T U)^T
    gram = ops.small_gram(Ut)                             # U^T U (segsum.hip)
    ST = _init_HT(K, G, None, dev, torch.float32, random_state, row_offset=col_offset)
    chunked_solve(ST, numerT, gram, chunk_size, chunk_max_iter, h_tol, l1_num=l1_reg, eps=epsilon)
    return ST.cpu().numpy()

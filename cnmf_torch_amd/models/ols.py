"""Gene spectra scores: OLS of (z-scored) expression on usages (C5, cnmf.py:56-126).

Beta = (X^T X)^{-1} X^T Y, no intercept, Y optionally z-scored column-wise with the
GLOBAL mean and ddof=0 std (variance floored at 1e-12, cnmf.py:90-96).  The reference
densifies each 1024-row batch of sparse Y to z-score it.  Here the z-scoring is done
algebraically on the accumulated products instead,

    X^T ((Y - 1 mu^T) / sd) = (X^T Y - (X^T 1) mu^T) / sd,

so sparse Y is never densified: X^T Y is a streamed sparse/dense product on the device,
accumulated in float64, and the tiny K x K system is solved by least squares.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

from .. import ops
from ..ops import sparse as sops
from .hvg import get_mean_var


def efficient_ols_all_cols(X, Y, batch_size: int = 1024, normalize_y: bool = False,
                           device=None):
    n, p = X.shape
    if Y.shape[0] != n:
        raise ValueError("X and Y must have the same number of rows.")
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if isinstance(Y, sops.DeviceCSR):
        dev = Y.device
    Xt = torch.as_tensor(np.asarray(X), dtype=torch.float64).to(dev)
    XtX = ops.small_gram(Xt)          # (segsum.hip; a library GEMM beyond 64 columns)
    if isinstance(Y, sops.DeviceCSR):     # resident CSR: one transposed-SpMM kernel pass
        XtY = sops.tspmm(Y, Xt).t()
    else:
        XtY = torch.zeros((p, Y.shape[1]), dtype=torch.float64, device=dev)
        step = max(int(batch_size), 1) * 16
        for a in range(0, n, step):
            b = min(n, a + step)
            blk = Y[a:b]
            if sp.issparse(blk):
                blk = blk.tocoo()
                idx = torch.as_tensor(np.vstack([blk.row, blk.col]), dtype=torch.long, device=dev)
                vals = torch.as_tensor(blk.data, dtype=torch.float64, device=dev)
                Yb = torch.sparse_coo_tensor(idx, vals, blk.shape, device=dev)
                XtY += torch.sparse.mm(Yb.t(), Xt[a:b]).t()
            else:
                Yb = torch.as_tensor(np.asarray(blk), dtype=torch.float64, device=dev)
                XtY += Xt[a:b].t() @ Yb
    if normalize_y:
        mean, var = get_mean_var(Y)
        var = np.array(var, dtype=np.float64)
        var[var < 1e-12] = 1e-12
        mu = torch.as_tensor(np.asarray(mean, dtype=np.float64), device=dev)
        sd = torch.sqrt(torch.as_tensor(var, device=dev))
        XtY = (XtY - Xt.sum(dim=0)[:, None] * mu[None, :]) / sd[None, :]
    beta = torch.linalg.lstsq(XtX.cpu(), XtY.cpu(), driver="gelsd").solution
    return beta.numpy()

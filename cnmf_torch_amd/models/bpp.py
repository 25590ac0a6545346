"""Exact non-negative least squares by block principal pivoting (nmf-torch ``algo='bpp'``;
SURVEY.md §2.3: nmf-torch's ANLS-BPP solver, not reachable from the reference CLI, which
fixes ``algo='mu'`` at cnmf.py:757-771).

Every NMF half-step of the Frobenius objective is, per column j, the quadratic program

    min_{x >= 0}  1/2 x^T G x - b_j^T x        (H step: G = W W^T, b = W x_j;
                                                 W step: G = A = sum h^T h, b = B_j)

which the MU / HALS kernels only approach iteratively.  Block principal pivoting
(Kim & Park, SIAM J. Sci. Comput. 33(6), 2011) finds its exact solution in a few
exchanges of the passive set F: solve G_FF x_F = b_F, set y = G x - b on the
complement, and swap every infeasible index (x_F < 0 or y_G < 0) -- with the
backup rule (only the largest infeasible index, after three exchanges that did not
shrink the infeasible set) that guarantees termination.

Batched form: all columns of all replicates are pivoted together.  A column's masked
system ``G o (F F^T) + diag(1 - F)`` is SPD whenever G is, so one batched LU
factorisation + solve per pivot round covers every column (float64; K <= 32 systems
are far below an MFMA tile, the batched LAPACK path is the right tool).  Columns that
are already feasible keep their solution.
"""
from __future__ import annotations

import torch


def nnls_bpp(G: torch.Tensor, B: torch.Tensor, l1: float = 0.0, l2: float = 0.0,
             max_rounds: int | None = None, col_chunk: int = 1 << 13) -> torch.Tensor:
    """Solve min_{x>=0} 1/2 x^T (G + l2 I) x - (b - l1)^T x for every column of ``B``.

    G: (R, K, K) symmetric PSD; B: (R, K, n).  Returns X (R, K, n) in B's dtype.  Columns
    are processed in chunks (at most ``col_chunk`` per replicate and 2^16 systems per
    chunk) to bound the (R, c, K, K) float64 workspace and the batched factorisations.
    """
    R, K, n = B.shape
    if G.shape != (R, K, K):
        raise ValueError(f"nnls_bpp: G {tuple(G.shape)} vs B {tuple(B.shape)}")
    out = torch.empty_like(B)
    eye = torch.eye(K, dtype=torch.float64, device=G.device)
    Gd = G.to(torch.float64)
    if l2:
        Gd = Gd + l2 * eye
    # a relative ridge keeps rank-deficient Grams (duplicate components) factorisable
    ridge = 1e-12 * Gd.diagonal(dim1=1, dim2=2).mean(dim=1).clamp_min(1e-300)
    Gd = Gd + ridge.view(R, 1, 1) * eye
    step = max(1, min(col_chunk, (1 << 16) // max(1, R)))
    for a in range(0, n, step):
        b = min(n, a + step)
        rhs = B[:, :, a:b].to(torch.float64).transpose(1, 2)         # (R, c, K)
        if l1:
            rhs = rhs - l1
        out[:, :, a:b] = _bpp_block(Gd, rhs, max_rounds).transpose(1, 2).to(B.dtype)
    return out


def _bpp_block(G: torch.Tensor, b: torch.Tensor, max_rounds: int | None) -> torch.Tensor:
    R, c, K = b.shape
    dev = b.device
    rounds = max_rounds if max_rounds is not None else 10 * K + 10
    F = torch.zeros((R, c, K), dtype=torch.bool, device=dev)          # passive set
    x = torch.zeros((R, c, K), dtype=torch.float64, device=dev)
    y = -b                                                             # gradient at x = 0
    alpha = torch.full((R, c), 3, dtype=torch.int32, device=dev)
    beta = torch.full((R, c), K + 1, dtype=torch.int32, device=dev)
    tol = 1e-12 * b.abs().amax(dim=2, keepdim=True).clamp_min(1e-300)
    Gc = G.unsqueeze(1)                                                # (R, 1, K, K)
    idx = torch.arange(K, device=dev)
    for _ in range(rounds):
        V = (F & (x < -tol)) | (~F & (y < -tol))
        nV = V.sum(dim=2, dtype=torch.int32)
        live = nV > 0
        if not bool(live.any()):
            break
        smaller = live & (nV < beta)
        beta = torch.where(smaller, nV, beta)
        alpha = torch.where(smaller, torch.full_like(alpha, 3), alpha)
        full = smaller | (live & (alpha >= 1))
        alpha = torch.where(live & ~smaller & (alpha >= 1), alpha - 1, alpha)
        # backup rule: exchange only the largest infeasible index
        last = torch.where(V, idx, torch.full_like(idx, -1)).amax(dim=2, keepdim=True)
        single = V & (idx == last)
        ex = torch.where(full.unsqueeze(2), V, single) & live.unsqueeze(2)
        F = F ^ ex
        Fm = F.to(torch.float64)
        A = Gc * (Fm.unsqueeze(3) * Fm.unsqueeze(2)) + torch.diag_embed(1.0 - Fm)
        rhs = (b * Fm).unsqueeze(3)
        sol, bad = _spd_solve(A.reshape(-1, K, K), rhs.reshape(-1, K, 1))
        if bool(bad.any()):
            # an fp32-accumulated Gram can be indefinite at the 1e-7 level: retry those
            # systems with a ridge of that size, in float64 on the host (rare)
            Ab = A.reshape(-1, K, K)[bad].cpu()
            rb = rhs.reshape(-1, K, 1)[bad].cpu()
            lift = 1e-6 * Ab.diagonal(dim1=1, dim2=2).abs().mean(dim=1).clamp_min(1e-300)
            Ab = Ab + lift.view(-1, 1, 1) * torch.eye(K, dtype=Ab.dtype)
            sol[bad] = (torch.linalg.pinv(Ab, hermitian=True) @ rb).squeeze(2).to(dev)
        sol = sol.view(R, c, K)
        sol = sol * Fm
        x = torch.where(live.unsqueeze(2), sol, x)
        yn = torch.einsum("rkl,rcl->rck", G, x) - b
        y = torch.where(live.unsqueeze(2), yn * (1.0 - Fm), y)
    return x.clamp_min(0.0)


def _spd_solve(A: torch.Tensor, rhs: torch.Tensor):
    """Batched LU solve of (m, K, K) SPD systems, at most 2^14 per factorisation call.
    Every solution is verified by its residual (on the GPU, batched Cholesky at large
    batch sizes returned garbage for some well-posed systems without flagging them).
    Returns the (m, K) solutions and a mask of systems that failed the check."""
    m, K = A.shape[0], A.shape[1]
    sol = torch.empty((m, K), dtype=A.dtype, device=A.device)
    bad = torch.zeros(m, dtype=torch.bool, device=A.device)
    step = 1 << 14
    for a in range(0, m, step):
        b = min(m, a + step)
        s, info = torch.linalg.solve_ex(A[a:b], rhs[a:b])
        s = s.squeeze(2)
        sol[a:b] = s
        # residual check: a factorisation that silently broke down leaves a large residual
        res = (A[a:b] @ s.unsqueeze(2) - rhs[a:b]).squeeze(2).abs().amax(dim=1)
        scale = rhs[a:b].squeeze(2).abs().amax(dim=1) + A[a:b].abs().amax(dim=(1, 2)) * \
            s.abs().amax(dim=1)
        bad[a:b] = (info != 0) | ~torch.isfinite(s).all(dim=1) | (res > 1e-8 * scale + 1e-300)
    return sol, bad


def objective_terms(x3: torch.Tensor, numer3: torch.Tensor, gram3: torch.Tensor):
    """Per-replicate <numer, x> and sum_j x_j^T G x_j (the solve kernels' lin/quad
    epilogue, used by the trace-trick loss)."""
    lin = (numer3 * x3).sum(dim=(1, 2))
    quad = (torch.bmm(gram3, x3) * x3).sum(dim=(1, 2))
    return lin, quad

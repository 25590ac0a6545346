"""PyTorch reference implementations of the native ops (CPU path + test oracle).

They implement exactly the contract of the HIP kernels (csrc/kernels/*.hip) in
vectorised torch, in whatever dtype they are given (float64 for the oracle).
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils.rng import philox_matrix


def _objective(X, N, G, l1, l2):
    """Block objective per replicate: sum x^T G x - 2 n.x + 2 l1 |x|_1 + l2 |x|^2."""
    q = (X * (torch.bmm(G, X) + l2 * X)).sum(dim=(1, 2))
    lin = (X * (N - l1)).sum(dim=(1, 2))
    return q - 2.0 * lin


def _step(algo, Xa, Na, Ga, l1_den, l2, eps):
    K = Xa.shape[1]
    if algo == 0:
        den = torch.bmm(Ga, Xa) + l2 * Xa + l1_den
        return torch.where(den < eps, torch.zeros_like(Xa), Xa * (Na / den))
    Xn = Xa.clone()
    for k in range(K):
        gx = torch.bmm(Ga[:, k:k + 1, :], Xn).squeeze(1)
        diag = (Ga[:, k, k] + l2).unsqueeze(1)
        old = Xn[:, k, :]
        upd = torch.clamp(old + (Na[:, k, :] - l1_den - gx - l2 * old) / diag, min=0.0)
        Xn[:, k, :] = torch.where(diag > eps, upd, old)
    return Xn


def solve(algo: int, x, numer, gram, rep_index, max_iter, tol, l1_num, l1_den, l2, eps,
          lin_out, quad_out, iters_out, nsplit=1, conv_mode=0, check_every=10,
          active=None) -> None:
    R, K, n = x.shape
    reps = (torch.arange(R, device=x.device) if rep_index is None
            else rep_index.to(device=x.device, dtype=torch.long))
    if active is not None:
        reps = reps[active.to(x.device)[reps] != 0]
    if reps.numel() == 0:
        return
    X = x[reps].clone()
    N = numer[reps].to(X.dtype)
    if l1_num > 0:
        N = torch.clamp(N - l1_num, min=0.0)
    G = gram[reps].to(X.dtype)
    m = reps.numel()
    active = torch.ones(m, dtype=torch.bool, device=x.device)
    iters = torch.zeros(m, dtype=torch.int32, device=x.device)
    check = nsplit <= 1
    loss_conv = check and conv_mode == 1
    every = max(1, int(check_every))
    f_prev = torch.zeros(m, dtype=X.dtype, device=x.device)
    have_prev = False
    it = 0
    while True:
        if loss_conv and it % every == 0:
            idx = torch.nonzero(active).flatten()
            if idx.numel() == 0:
                break
            f = _objective(X[idx], N[idx], G[idx], l1_den, l2)
            if have_prev:
                conv = torch.abs(f_prev[idx] - f) <= tol * torch.abs(f_prev[idx])
                active[idx[conv]] = False
            f_prev[idx] = f
            have_prev = True
        if it >= int(max_iter):
            break
        idx = torch.nonzero(active).flatten()
        if idx.numel() == 0:
            break
        Xa = X[idx]
        Xn = _step(algo, Xa, N[idx], G[idx], l1_den, l2, eps)
        X[idx] = Xn
        iters[idx] += 1
        it += 1
        if check and not loss_conv:
            d2 = ((Xn - Xa) ** 2).sum(dim=(1, 2))
            x2 = (Xa ** 2).sum(dim=(1, 2))
            conv = torch.sqrt(d2) / (torch.sqrt(x2) + eps) < tol
            active[idx[conv]] = False
    x[reps] = X
    if lin_out is not None or quad_out is not None:
        lin = (numer[reps].to(X.dtype) * X).sum(dim=(1, 2))
        quad = (X * torch.bmm(G, X)).sum(dim=(1, 2))
        if lin_out is not None:
            lin_out[reps] = lin.to(lin_out.dtype)
        if quad_out is not None:
            quad_out[reps] = quad.to(quad_out.dtype)
    if iters_out is not None:
        iters_out[reps] += iters.to(iters_out.dtype)


def philox_fill(out: torch.Tensor, seeds, scales, stream: int, mode: int = 0,
                row_offset: int = 0) -> None:
    R, rows, cols = out.shape
    seeds = [int(s) for s in torch.as_tensor(seeds).cpu().tolist()]
    scales = torch.as_tensor(scales, dtype=torch.float32).cpu()
    for r in range(R):
        m = torch.from_numpy(philox_matrix(seeds[r], stream, rows, cols, mode, row_offset))
        out[r].copy_((m * scales[r]).to(out.dtype))


def conv_update(lin, quad, x_sq, state, n, pass_idx, tol, final, init=False):
    e = torch.sqrt(torch.clamp(x_sq - 2.0 * lin[:n].double() + quad[:n].double(), min=0.0))
    e = e.to(state["err"].device)
    if init:
        for k in ("err_init", "err_prev", "err"):
            state[k][:n] = e
        state["active"][:n] = 1
        state["converged"][:n] = 0
        state["n_pass"][:n] = 0
        return
    act = state["active"][:n] != 0
    state["err"][:n] = torch.where(act, e, state["err"][:n])
    state["n_pass"][:n] = torch.where(act, torch.full_like(state["n_pass"][:n], pass_idx),
                                      state["n_pass"][:n])
    rel = (state["err_prev"][:n] - e) / torch.clamp(state["err_init"][:n], min=1e-300)
    conv = act & (rel < tol)
    stop = conv | (act & bool(final))
    state["converged"][:n] = torch.where(conv, torch.ones_like(state["converged"][:n]),
                                         state["converged"][:n])
    keep = act & ~stop
    state["err_prev"][:n] = torch.where(keep, e, state["err_prev"][:n])
    state["active"][:n] = torch.where(stop, torch.zeros_like(state["active"][:n]),
                                      state["active"][:n])

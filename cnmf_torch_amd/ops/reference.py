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


def conv_update(lin, quad, x_sq, state, n, pass_idx, tol, final, init=False, max_pass=0):
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
    new_pass = (torch.full_like(state["n_pass"][:n], pass_idx) if pass_idx >= 0
                else state["n_pass"][:n] + 1)              # pass_idx < 0: count passes
    state["n_pass"][:n] = torch.where(act, new_pass, state["n_pass"][:n])
    rel = (state["err_prev"][:n] - e) / torch.clamp(state["err_init"][:n], min=1e-300)
    conv = act & (rel < tol)
    over = (new_pass >= max_pass) if max_pass > 0 else torch.zeros_like(act)
    stop = conv | (act & (bool(final) | over))
    state["converged"][:n] = torch.where(conv, torch.ones_like(state["converged"][:n]),
                                         state["converged"][:n])
    keep = act & ~stop
    state["err_prev"][:n] = torch.where(keep, e, state["err_prev"][:n])
    state["active"][:n] = torch.where(stop, torch.zeros_like(state["active"][:n]),
                                      state["active"][:n])


def beta_terms(X: torch.Tensor, P: torch.Tensor, beta: float, eps: float):
    """Q = X * P^(beta-2), D = P^(beta-1) with P clamped at eps (beta_mu.hip)."""
    Pc = torch.clamp(P, min=eps)
    if beta == 1.0:
        return X / Pc, None
    if beta == 0.0:
        r = Pc.reciprocal()
        return X * r * r, r
    return X * Pc ** (beta - 2.0), Pc ** (beta - 1.0)


def beta_loss_terms(X: torch.Tensor, P: torch.Tensor, beta: float, eps: float) -> torch.Tensor:
    Pc = torch.clamp(P, min=eps)
    if beta == 1.0:
        pos = X > 0
        t = torch.where(pos, X * torch.log(torch.where(pos, X, torch.ones_like(X)) / Pc),
                        torch.zeros_like(Pc))
        return t - X + Pc
    if beta == 0.0:
        d = torch.clamp(X / Pc, min=eps)
        return d - torch.log(d) - 1.0
    return (X ** beta + (beta - 1.0) * Pc ** beta - beta * X * Pc ** (beta - 1.0)) / (
        beta * (beta - 1.0))


def beta_contract(side: int, X, HT3, W3, beta: float, eps: float, want_num: bool = True,
                  want_loss: bool = False, active=None, row_chunk: int = 4096):
    """Reference of cnmf_beta_contract: returns (num, den, loss) with num/den (R,K,N) for
    side 0 (H) and (R,K,G) for side 1 (W); den is None for beta == 1; loss (R,) float64
    (side 0 only) or None.  Inactive replicates get zeros."""
    R, K, N = HT3.shape
    G = W3.shape[2]
    dt = HT3.dtype
    out_n = N if side == 0 else G
    num = torch.zeros((R, K, out_n), dtype=dt, device=HT3.device) if want_num else None
    den = (torch.zeros((R, K, out_n), dtype=dt, device=HT3.device)
           if (want_num and beta != 1.0) else None)
    loss = torch.zeros(R, dtype=torch.float64, device=HT3.device) if (want_loss and side == 0) else None
    reps = range(R) if active is None else [r for r in range(R) if int(active[r]) != 0]
    for r in reps:
        for a in range(0, N, row_chunk):
            b = min(N, a + row_chunk)
            x = X[a:b].to(dt)
            h = HT3[r, :, a:b]                      # (K, c)
            P = h.t() @ W3[r]                       # (c, G)
            Q, D = beta_terms(x, P, beta, eps)
            if want_num:
                if side == 0:
                    num[r, :, a:b] = W3[r] @ Q.t()
                    if D is not None:
                        den[r, :, a:b] = W3[r] @ D.t()
                else:
                    num[r] += h @ Q
                    if D is not None:
                        den[r] += h @ D
            if loss is not None:
                loss[r] += beta_loss_terms(x.double(), P.double(), beta, eps).sum()
    return num, den, loss


def beta_update_h(X, HT3, W3, beta, eps, l1=0.0, l2=0.0, gamma=1.0, act=None, tol=None,
                  iters=None, conv_mode=0, check_every=10, hstate=None, contract=None):
    """Reference of the fused in-place usage update (beta_mu.hip, upd != 0).  ``contract``:
    the beta_contract implementation to use (ops: the rank-general native one)."""
    beta_contract_ = contract or beta_contract
    R = HT3.shape[0]
    loss_rule = tol is not None and conv_mode == 1
    num, den, f = beta_contract_(0, X, HT3, W3, beta, eps, True, loss_rule, act)
    if den is None:
        den = W3.sum(dim=2, keepdim=True)
    d = den + l1 + l2 * HT3
    d = torch.where(d == 0, torch.full_like(d, eps), d)
    delta = num / d
    if gamma != 1.0:
        delta = delta ** gamma
    live = torch.ones(R, dtype=torch.bool, device=HT3.device) if act is None else (act[:R] != 0)
    delta = torch.where(live.view(R, 1, 1), delta, torch.ones_like(delta))
    if tol is not None and not loss_rule:
        dn = torch.linalg.vector_norm((HT3 * (delta - 1.0)).double(), dim=(1, 2))
        hn = torch.linalg.vector_norm(HT3.double(), dim=(1, 2))
    HT3.mul_(delta)
    if tol is not None:
        if loss_rule:
            hs = hstate.view(-1, 2)[:R]
            f = f.to(hs.device)
            steps = hs[:, 1].long()
            every = max(1, int(check_every))
            at_check = live & (steps % every == 0)
            conv = at_check & (steps > 0) & ((hs[:, 0] - f).abs() <= tol * hs[:, 0].abs())
            hs[:, 0] = torch.where(at_check, f, hs[:, 0])
            hs[:, 1] = torch.where(live, hs[:, 1] + 1, hs[:, 1])
            stop = conv
        else:
            stop = live & (dn / (hn + eps) < tol)
        act[:R][stop] = 0
        if iters is not None:
            iters[:R] += live.to(iters.dtype)


def beta_h_block(X, HT3, W3, beta, eps, nsteps, l1=0.0, l2=0.0, gamma=1.0, act=None, tol=None,
                 iters=None, conv_mode=1, hstate=None, loss_entry=False, contract=None):
    """Reference of the multi-step usage solve block (beta_planes.hip, side 0): ``nsteps``
    MU steps of the live replicates, then the stopping rule: conv_mode 1 compares the
    block's exit objective -- the beta-divergence at the iterate its last step starts from
    (after the block for a one-step block) -- with the previous one (``loss_entry``: the
    objective before the block, evaluated here; else the value ``hstate`` recorded);
    conv_mode 0 reads the relative change of the block's last step."""
    beta_contract_ = contract or beta_contract
    R = HT3.shape[0]
    live = torch.ones(R, dtype=torch.bool, device=HT3.device) if act is None else (act[:R] != 0)
    rule = tol is not None
    f_entry = None
    if rule and conv_mode == 1 and loss_entry and nsteps > 0:
        f_entry = beta_contract_(0, X, HT3, W3, beta, eps, False, True, act)[2].to(HT3.device)
    dn = hn = None
    f_exit = None
    exit_in_last = nsteps >= 2
    for s in range(nsteps):
        # the kernel reads the exit objective off the last step's P pass (here: the same
        # contraction returns it)
        at_exit = rule and conv_mode == 1 and exit_in_last and s == nsteps - 1
        num, den, f = beta_contract_(0, X, HT3, W3, beta, eps, True, at_exit, act)
        if at_exit:
            f_exit = f.to(HT3.device)
        if den is None:
            den = W3.sum(dim=2, keepdim=True)
        d = den + l1 + l2 * HT3
        d = torch.where(d == 0, torch.full_like(d, eps), d)
        delta = num / d
        if gamma != 1.0:
            delta = delta ** gamma
        delta = torch.where(live.view(R, 1, 1), delta, torch.ones_like(delta))
        if s == nsteps - 1 and rule and conv_mode == 0:
            dn = torch.linalg.vector_norm((HT3 * (delta - 1.0)).double(), dim=(1, 2))
            hn = torch.linalg.vector_norm(HT3.double(), dim=(1, 2))
        HT3.mul_(delta)
    if not rule:
        return
    if conv_mode == 1:
        if f_exit is None:
            f_exit = beta_contract_(0, X, HT3, W3, beta, eps, False, True, act)[2].to(HT3.device)
        hs = hstate.view(-1, 2)[:R]
        f_prev = f_entry if loss_entry else hs[:, 0]
        checked = torch.full_like(live, bool(loss_entry)) | (hs[:, 1] > 0)
        stop = live & checked & ((f_prev - f_exit).abs() <= tol * f_prev.abs())
        hs[:, 0] = torch.where(live, f_exit, hs[:, 0])
        hs[:, 1] = torch.where(live, hs[:, 1] + 1, hs[:, 1])
    elif nsteps > 0:
        stop = live & (dn / (hn + eps) < tol)
    else:
        stop = torch.zeros_like(live)
    act[:R][stop] = 0
    if iters is not None:
        iters[:R] += live.to(iters.dtype) * int(nsteps)


def beta_w_update(W3, num, den, hsum, An, Ad, an_out, dn_out, beta, gamma, l1, l2, eps, tol,
                  act, iters=None):
    """Reference of the anchored online spectra step (beta_mu.hip beta_w_update_kernel)."""
    R = W3.shape[0]
    live = act[:R] != 0
    if not bool(live.any()):
        return
    nu = num.sum(0)
    kl = beta == 1.0
    dn = hsum.unsqueeze(2).expand_as(nu) if kl else den.sum(0)
    ad = Ad.unsqueeze(2) if kl else Ad
    an = W3 ** (1.0 / gamma) * nu
    B = ad + dn + l1 + l2 * W3
    B = torch.where(B == 0, torch.full_like(B, eps), B)
    Wn = ((An + an) / B) ** gamma
    m = live.view(R, 1, 1)
    d = torch.linalg.vector_norm(torch.where(m, Wn - W3, 0).double(), dim=(1, 2))
    o = torch.linalg.vector_norm(W3.double(), dim=(1, 2))
    W3.copy_(torch.where(m, Wn, W3))
    an_out.copy_(torch.where(m, an, an_out))
    if not kl:
        dn_out.copy_(torch.where(m, dn, dn_out))
    stop = live & (d / (o + eps) < tol)
    act[:R][stop] = 0
    if iters is not None:
        iters[:R] += live.to(iters.dtype)


def _bf16_rn_bits(v: torch.Tensor) -> torch.Tensor:
    """Round-to-nearest-even bf16 bit patterns (int32 holding 16 bits) of finite fp32."""
    u = v.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return (u & 0xFFFF).to(torch.int32)


def _bits_to_f32(h: torch.Tensor) -> torch.Tensor:
    return (h.to(torch.int64) << 16).to(torch.int32).view(torch.float32)


def split_planes(S: torch.Tensor, nplanes: int, ld: int) -> torch.Tensor:
    """(nplanes, rows, ld) int16 bf16 planes of fp32 S (columns beyond S are zero)."""
    rows, cols = S.shape
    out = torch.zeros((nplanes, rows, ld), dtype=torch.int16, device=S.device)
    r = S.to(torch.float32)
    for p in range(nplanes):
        h = _bf16_rn_bits(r)
        out[p, :, :cols] = h.to(torch.int16)   # wraps to the same 16-bit pattern
        r = r - _bits_to_f32(h)
    return out


def planes_to_f64(P: torch.Tensor) -> torch.Tensor:
    """bf16 planes (P, rows, k) int16 -> their float64 values, per plane."""
    return _bits_to_f32(P.to(torch.int32) & 0xFFFF).to(torch.float64)


def gemm_planes(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """sum_{i + j <= 2} A_i B_j^T in float64 (oracle of ops.gemm_planes)."""
    Af, Bf = planes_to_f64(A), planes_to_f64(B)
    out = torch.zeros((A.shape[1], B.shape[1]), dtype=torch.float64, device=A.device)
    for i in range(A.shape[0]):
        for j in range(B.shape[0]):
            if i + j <= 2:
                out += Af[i] @ Bf[j].t()
    return out


def colstats(X: torch.Tensor):
    inf = torch.tensor(float("inf"), dtype=X.dtype, device=X.device)
    mn = torch.where(X > 0, X, inf).amin(0) if X.shape[0] else \
        torch.full((X.shape[1],), float("inf"), dtype=X.dtype, device=X.device)
    sq = (X.to(torch.float64) ** 2).sum(0)
    neg = (X < 0).any(0).to(torch.int32)
    return mn, sq, neg


def count_unit_check(X: torch.Tensor, mn: torch.Tensor) -> torch.Tensor:
    bad = torch.zeros(X.shape[1], dtype=torch.int32, device=X.device)
    ok_col = (mn > 0) & torch.isfinite(mn)
    for d in range(1, 9):
        c = X / (mn / d)
        off = ((c - torch.round(c)).abs() > 4e-7 * c + 1e-4) | (c >= 65535.5)
        off &= X != 0
        bad |= (off.any(0) & ok_col).to(torch.int32) << (d - 1)
    return bad

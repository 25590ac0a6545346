"""The rank-general GPU paths: Frobenius MU at any K, HALS to 512 and the beta-divergence
MU beyond the panel kernels (csrc/kernels/solve_any.hip, beta_any.hip).  At those ranks
the sweep's products are real GEMMs and run as batched library GEMMs; everything around
them -- updates, objectives, stop decisions, the beta terms -- is HIP.  Entered from
ops.solve and the ops.beta_* wrappers (the reference's -k is
unbounded, cnmf.py:1416-1417)."""
from __future__ import annotations

import torch

from . import ALGO_MU, _gram_op, _hip, _stream_ptr, beta_mode


def solve_any_k(algo: int, K: int) -> bool:
    """Whether a rank-K solve runs the rank-general kernels (solve_any.hip): K beyond the
    register-tiled instantiations -- MU K > 128 or not an instantiated rank, HALS K > 64."""
    if _hip is None:
        return False
    return (not _hip.solve_native_k(K)) or (K > 64 and algo != ALGO_MU)


def solve_any_max_k(algo: int) -> int | None:
    """Largest K the rank-general solve takes (None: any -- MU's sweep is a library GEMM
    plus elementwise kernels; HALS keeps a 64-column tile of every component in LDS)."""
    return None if algo == ALGO_MU else int(_hip.solve_any_hals_max_k())


def _solve_any(a, x, numer, gram, rep_index, max_iter, tol, l1_num, l1_den, l2, eps,
               lin_out, quad_out, iters_out, nsplit, conv_mode, check_every, active) -> None:
    """ops.solve at any K (csrc/kernels/solve_any.hip; contract = reference.solve): per
    sweep D = Gram x is one batched library GEMM (torch.bmm -> rocBLAS / hipBLASLt), the
    objective / update / stop decisions are HIP kernels with device-side live flags.  The
    host looks at the flags once per objective check (outside graph capture) to end the
    loop when every replicate has stopped."""
    h = _hip
    R, K, n = x.shape
    mk = solve_any_max_k(a)
    if mk is not None and K > mk:
        raise ValueError(f"solve: HALS at K={K} exceeds the rank-general kernel's maximum {mk} "
                         "(use algo='mu' or 'bpp')")
    for name, t in (("x", x), ("numer", numer)):
        if t.dtype != torch.float32 or (n > 1 and t.stride(2) != 1):
            raise ValueError(f"solve: {name} must be float32 with unit column stride")
    dev = x.device
    st = _stream_ptr(x)
    ident = rep_index is None
    reps = None if ident else rep_index.to(device=dev, dtype=torch.int32).contiguous()
    m = R if ident else int(reps.numel())
    if m == 0 or n == 0:
        return
    reps_l = None if ident else reps.long()
    act = torch.ones(m, dtype=torch.int32, device=dev)
    if active is not None:
        act = (active[:R] if ident else active[reps_l]).ne(0).to(torch.int32)
    act0 = act.clone()
    G = gram.contiguous()
    Gm = G if ident else G.index_select(0, reps_l)
    D = torch.empty((m, K, n), dtype=torch.float32, device=dev)

    def gram_x():
        torch.bmm(Gm, x if ident else x.index_select(0, reps_l), out=D)

    per = max(256, -(-n // max(1, min(-(-n // 256), 2048 // m))))
    nblk_s = -(-n // per)
    nblk_h = -(-n // 64)
    part = torch.empty(m * max(nblk_s, nblk_h) * 2, dtype=torch.float64, device=dev)
    f_prev = torch.zeros(m, dtype=torch.float64, device=dev)
    it_ptr = iters_out.data_ptr() if iters_out is not None else 0
    if iters_out is not None and (iters_out.dtype != torch.int32 or not iters_out.is_contiguous()):
        raise ValueError("iters_out: contiguous int32")
    rp = reps.data_ptr() if reps is not None else 0

    def launch(op):
        h.solve_any(op, x.data_ptr(), x.stride(0), x.stride(1), numer.data_ptr(), numer.stride(0),
                    numer.stride(1), D.data_ptr(), G.data_ptr(), K * K, rp, act.data_ptr(), m, K,
                    n, per, float(l1_num), float(l1_den), float(l2), float(eps), part.data_ptr(),
                    it_ptr if op >= 2 else 0, st)

    def decide(mode, nblk, have_prev=0, lin=None, quad=None):
        h.solve_any_conv(mode, part.data_ptr(), nblk, m, act.data_ptr(), act0.data_ptr(), rp,
                         f_prev.data_ptr(), int(have_prev), float(tol), float(eps),
                         lin.data_ptr() if lin is not None else 0,
                         quad.data_ptr() if quad is not None else 0, st)

    check = nsplit <= 1
    loss_conv = check and conv_mode == 1
    every = max(1, int(check_every))
    capturing = torch.cuda.is_current_stream_capturing()
    have_prev = False
    it = 0
    while True:
        fresh = False
        if loss_conv and it % every == 0:
            if it > 0 and not capturing and not bool(act.any()):
                break
            gram_x()
            fresh = True
            launch(0)
            decide(0, nblk_s, have_prev)
            have_prev = True
        if it >= int(max_iter):
            break
        if check and not loss_conv and it > 0 and it % every == 0 and not capturing \
                and not bool(act.any()):
            break
        if a == ALGO_MU:
            if not fresh:
                gram_x()
            launch(3 if (check and not loss_conv) else 2)
        else:
            launch(5 if (check and not loss_conv) else 4)
        it += 1
        if check and not loss_conv:
            decide(1, nblk_s if a == ALGO_MU else nblk_h)
    if lin_out is not None or quad_out is not None:
        for name, t in (("lin_out", lin_out), ("quad_out", quad_out)):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
                raise ValueError(f"{name}: contiguous float32")
        gram_x()
        launch(1)
        decide(2, nblk_s, lin=lin_out, quad=quad_out)


def beta_any_k(K: int, beta: float) -> bool:
    """Whether the beta-MU ops run rank K on the rank-general path (beta_any.hip): beyond
    the split-bf16 panel kernels -- KL K > 64, IS / general beta K > 56 (an IS K = 64 panel
    pair exceeds the LDS)."""
    if _hip is None:
        return False
    return K > (int(_hip.bp_max_k()) if beta == 1.0 else 56)


def _beta_contract_any(side: int, X: torch.Tensor, HT3: torch.Tensor, W3: torch.Tensor,
                       beta: float, eps: float, want_num: bool = True, want_loss: bool = False,
                       active: torch.Tensor | None = None):
    """reference.beta_contract's contract at any K on the GPU: per block of rows, P =
    H^T W and the numerator / denominator contractions are batched library GEMMs (real
    GEMMs at these ranks), Q = X p^(beta-2), D = p^(beta-1) and the divergence sums one
    pass of beta_any_terms (csrc/kernels/beta_any.hip) over P, in place."""
    R, K, N = HT3.shape
    G = W3.shape[2]
    dev = HT3.device
    mode = beta_mode(beta)
    out_n = N if side == 0 else G
    num = torch.zeros((R, K, out_n), dtype=torch.float32, device=dev) if want_num else None
    den = (torch.zeros((R, K, out_n), dtype=torch.float32, device=dev)
           if (want_num and mode != 0) else None)
    loss = (torch.zeros(R, dtype=torch.float64, device=dev) if (want_loss and side == 0)
            else None)
    act = None if active is None else active[:R].to(torch.int32).contiguous()
    Xf = X if (X.dtype == torch.float32 and X.stride(-1) == 1) else X.float().contiguous()
    Wf = W3.float()
    rows = int(_hip.beta_any_rows())
    c = max(rows, min(N, (1 << 28) // max(1, R * G)))     # <= 1 GiB of P per block
    st = _stream_ptr(HT3)
    for a in range(0, N, c):
        b = min(N, a + c)
        h = HT3[:, :, a:b].float()
        P = torch.bmm(h.transpose(1, 2), Wf)            # (R, c, G)
        Dm = torch.empty_like(P) if den is not None else None
        part = (torch.empty((R, -(-(b - a) // rows)), dtype=torch.float64, device=dev)
                if loss is not None else None)
        _hip.beta_any_terms(mode, Xf[a:b].data_ptr(), Xf.stride(0), P.data_ptr(),
                            Dm.data_ptr() if Dm is not None else 0, R, b - a, G, float(beta),
                            float(eps), act.data_ptr() if act is not None else 0,
                            int(bool(want_num)), part.data_ptr() if part is not None else 0, st)
        if want_num:
            if side == 0:
                num[:, :, a:b] = torch.bmm(Wf, P.transpose(1, 2))
                if Dm is not None:
                    den[:, :, a:b] = torch.bmm(Wf, Dm.transpose(1, 2))
            else:
                num.baddbmm_(h, P)
                if Dm is not None:
                    den.baddbmm_(h, Dm)
        if part is not None:
            loss += part.sum(1)
    return num, den, loss

"""NMFBatchSolver: beta-divergence (KL / IS / general beta) MU: split-bf16 usage kernels,
anchored online spectra update (split out of models/nmf.py)."""
from __future__ import annotations

import os

import torch

from .. import ops
from .nmf_base import _count_units
from .nmf_batch import _Batch, _PassPipeline


class _BetaMixin:
    """NMFBatchSolver methods: beta-divergence (KL / IS / general beta) MU: split-bf16
    usage kernels, anchored online spectra update."""

    # ------------------------------------------------------------------ beta-divergence MU
    def _beta_gamma(self) -> float:
        b = self.beta
        if b < 1:
            return 1.0 / (2.0 - b)
        if b > 2:
            return 1.0 / (b - 1.0)
        return 1.0

    def _mu_apply(self, x3: torch.Tensor, num: torch.Tensor, den: torch.Tensor, l1: float,
                  l2: float, mask: torch.Tensor | None = None) -> None:
        """x3 *= ((num / (den + l1 + l2 x3)) ** gamma) in place (sklearn's MU update with the
        zero-denominator guard); ``mask`` (R,1,1 bool) leaves other replicates untouched."""
        eps = self.opts.eps
        d = den + l1 if l2 == 0.0 else den + l1 + l2 * x3
        d = torch.where(d == 0, torch.full_like(d, eps), d)
        delta = num / d
        g = self._beta_gamma()
        if g != 1.0:
            delta = delta.pow_(g)
        if mask is not None:
            delta = torch.where(mask, delta, torch.ones_like(delta))
        x3.mul_(delta)

    def _xt(self) -> torch.Tensor | None:
        """X^T (G, N), leading dimension padded to a multiple of 4 (float4 loads), for the
        W-side beta kernel (beta_planes.hip reads X along cells there); GPU only.  None
        when a second copy of X would not fit next to it (e.g. the 200 GB 10M x 5k matrix
        on one 288 GB GPU): the spectra side then runs the first-generation kernel
        (beta_mu.hip), which reads X in place."""
        if self.X.device.type != "cuda" or self._XT is False:
            return None
        if self._XT is None:
            N, G = self.X.shape
            need = G * (-(-N // 4) * 4) * self.X.element_size()
            free, _ = torch.cuda.mem_get_info(self.X.device)
            if need > 0.5 * free:
                self._XT = False
                return None
            buf = torch.zeros((G, -(-N // 4) * 4), device=self.X.device, dtype=self.X.dtype)
            buf[:, :N] = self.X.t()
            self._XT = buf[:, :N]
        return self._XT

    def _kl_sparse(self):
        """CSR of X (ops.KLCSR) when the KL MU statistics run on the sparse kernels
        (sparse_kl.hip): KL on the native GPU path with X at most ``kl_sparse_density``
        non-zero (``CNMF_KL_SPARSE=1`` forces it, ``=0`` disables it); else None (dense
        split-precision kernels).  Decided once per solver (one host sync)."""
        if getattr(self, "_beta_K", 0) > 32:     # the CSR kernels stop at K = 32
            return None
        if "_kl_csr" in self.__dict__:
            return self._kl_csr
        csr = None
        X = self.X
        env = os.environ.get("CNMF_KL_SPARSE", "")
        if (self.beta == 1.0 and env != "0" and isinstance(X, torch.Tensor)
                and X.device.type == "cuda" and X.dtype == torch.float32
                and self.opts.n_components <= 32 and ops.use_native(X)):
            dens = float((X != 0).sum()) / max(X.numel(), 1)
            if env == "1" or dens <= float(self.opts.kl_sparse_density):
                csr = ops.kl_csr(X)
        self._kl_csr = csr
        self._kl_csrT = {}
        return csr

    def _kl_counts(self):
        """(xh (N, G) float16, xth (G, N) float16, unit (G,), 1 / unit (G,)) when the dense
        KL kernels read X as fp16 counts: cNMF's normalised counts are integer counts over
        a per-gene std (X == C u_g, _count_units), and counts <= 2048 are exact in fp16.
        Half the bytes of the per-step X re-reads that bound those kernels
        (profiles/r3m_*), and xth replaces the fp32 X^T copy.  None for other data, the
        sparse path.  Only the spectra side reads the fp16 counts, the usage side fp32 X
        -- on the usage side the fp16 -> fp32 conversion costs more issue than the halved
        bytes save (326-329 vs 314-317 rep/s with both sides, profiles/r3v_*, r3w_*)."""
        if "_klc" in self.__dict__:
            return self._klc
        res = None
        X = self.X
        if (self.beta == 1.0 and isinstance(X, torch.Tensor) and X.device.type == "cuda"
                and X.dtype == torch.float32 and ops.use_native(X)
                and self._kl_sparse() is None):
            unit = _count_units(X, self._colstats)
            if unit is not None:
                unit = unit.to(device=X.device, dtype=torch.float32).contiguous()
                C = torch.round(X / unit)
                if float(C.max()) <= 2048.0:
                    N, G = X.shape
                    xh = C.to(torch.float16)
                    Np = -(-N // 4) * 4               # 8-byte rows: fp16 x4 loads
                    xth = torch.zeros((G, Np), dtype=torch.float16, device=X.device)
                    xth[:, :N] = xh.t()
                    res = (xh, xth[:, :N], unit, (1.0 / unit).contiguous())
                del C
        self._klc = res
        return res

    def _kl_rows_T(self, a: int, b: int):
        """Tiled CSRs of X[a:b]^T (genes x chunk cells) for the sparse spectra numerators."""
        key = (a, b)
        if key not in self._kl_csrT:
            self._kl_csrT[key] = ops.kl_csr_tiles(self.X[a:b], self._beta_K or self.opts.n_components)
        return self._kl_csrT[key]

    def _beta_w_partials(self, xc, xtc, H3c, W3, active, panels=None, rows=None):
        """(splits, R, K, G) W-side partials: the sparse KL kernel over X[rows]^T, the
        split-bf16 kernel through X^T, or the fp32 kernel reading X in place when X^T is
        not kept (see _xt)."""
        if rows is not None and self._kl_sparse() is not None:
            return ops.kl_sparse_w_num(self._kl_rows_T(*rows), H3c, W3, self.opts.eps,
                                       active=active, st=panels), None
        klc = self._kl_counts() if rows is not None else None
        if klc is not None:
            a, b = rows
            return ops.beta_w_partials(xc, None, H3c, W3, self.beta, self.opts.eps,
                                       active=active, panels=panels, xth=klc[1][:, a:b],
                                       unit_inv=klc[3])
        if xc.device.type == "cuda" and xtc is None:
            num, den, _ = ops.beta_contract("w", xc, H3c, W3, self.beta, self.opts.eps,
                                            active=active, reduce=False)
            return num, den
        return ops.beta_w_partials(xc, xtc, H3c, W3, self.beta, self.opts.eps, active=active,
                                   panels=panels)

    def _chunk_xsum(self, xc: torch.Tensor) -> float:
        """sum(X) of a row block in float64 (the KL objective's linear term), cached per
        block: X never changes, so this host sync happens once per block per solver."""
        key = (xc.data_ptr(), tuple(xc.shape))
        cache = self.__dict__.setdefault("_xsum_cache", {})
        if key not in cache:
            cache[key] = float(xc.sum(dtype=torch.float64))
        return cache[key]

    def _beta_panels(self, F3: torch.Tensor):
        """Kernel operand of a factor that stays fixed over the next kernel launches: its
        split-bf16 panels, or its padded transpose for the sparse KL kernels (GPU only; the
        CPU reference works on the fp32 factor directly)."""
        if F3.device.type != "cuda":
            return None
        if self._kl_sparse() is not None:
            return ops.kl_st(F3)
        return ops.beta_panels(F3, self.beta)

    def _beta_h_update(self, xc, H3c, W3, l1, l2, act=None, panels=None, rows=None):
        """One fused MU step of the usages H3c (R, K, c) in place against W3 on rows xc
        (replicates with act == 0 untouched)."""
        csr = self._kl_sparse() if rows is not None else None
        if csr is not None:
            ops.kl_sparse_h_block(ops.kl_csr_rows(csr, *rows), H3c, W3, self.opts.eps, 1, l1,
                                  l2, act=act, st=panels)
            return
        ops.beta_h_block(xc, H3c, W3, self.beta, self.opts.eps, 1, l1, l2, self._beta_gamma(),
                         act=act, panels=panels)

    def _beta_h_solve(self, xc, hc, W3, act, iters, wpan=None, block: int = 8,
                      rows=None) -> None:
        """Inner usage loop of one chunk: up to ``online_chunk_max_iter`` fused MU steps.
        With ``online_inner_conv='loss'`` (default) one launch runs ``inner_check_every``
        steps, and the block objective -- the chunk's beta-divergence after the block
        against the one before it -- stops a replicate once it changed by <=
        ``online_h_tol`` (relative; the Frobenius solve's conv_mode-1 rule, checked every
        ``inner_check_every`` steps); else one step per launch on the relative iterate
        change.  The rule runs on the device; whether anybody is still active is read from
        a pinned copy one launch group late, so the GPU always has work queued and the host
        never drains the stream (launches for finished replicates exit at once)."""
        o = self.opts
        W3 = W3.contiguous() if W3.stride(-1) != 1 else W3
        cuda = xc.device.type == "cuda"
        den_vec = (W3.sum(dim=2, dtype=torch.float32).contiguous()
                   if self.beta == 1.0 and cuda else None)
        csr = self._kl_sparse() if (cuda and rows is not None) else None
        klc = None      # the usage side reads fp32 X (see _kl_counts)
        if cuda and wpan is None:
            wpan = ops.kl_st(W3) if csr is not None else ops.beta_panels(W3, self.beta)
        cmode = 1 if o.online_inner_conv == "loss" else 0
        per = max(1, int(o.inner_check_every)) if cmode == 1 else 1
        group = 1 if cmode == 1 else block
        hstate = torch.zeros((W3.shape[0], 2), dtype=torch.float64, device=xc.device)
        xsum = self._chunk_xsum(xc) if (cuda and self.beta == 1.0 and cmode == 1) else None
        max_it = int(o.online_chunk_max_iter)
        pending = None
        it = 0
        first = True
        while it < max_it:
            for _ in range(group):
                if it >= max_it:
                    break
                m = min(per, max_it - it)
                if csr is not None:
                    ops.kl_sparse_h_block(ops.kl_csr_rows(csr, *rows), hc, W3, o.eps, m,
                                          o.l1_H, o.l2_H, act=act, tol=o.online_h_tol,
                                          iters=iters, conv_mode=cmode, hstate=hstate,
                                          loss_entry=first, den_vec=den_vec, st=wpan,
                                          xsum=xsum)
                else:
                    ops.beta_h_block(xc, hc, W3, self.beta, o.eps, m, o.l1_H, o.l2_H,
                                     self._beta_gamma(), act=act, tol=o.online_h_tol,
                                     iters=iters, conv_mode=cmode, hstate=hstate,
                                     loss_entry=first, den_vec=den_vec, panels=wpan,
                                     xsum=xsum,
                                     xh=klc[0][rows[0]:rows[1]] if klc is not None else None,
                                     unit=klc[2] if klc is not None else None)
                first = False
                it += m
            if not cuda:
                if int(act.sum()) == 0:
                    break
                continue
            flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
            flag.copy_(act.max().view(1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            prev, pending = pending, (ev, flag)
            if prev is not None:
                prev[0].synchronize()
                if int(prev[1][0]) == 0:
                    break

    def _beta_w_stats(self, xc, H3c, W3, xtc=None, active=None, rows=None):
        """(num, den) W-side MU statistics of rows xc (den broadcastable to (R,K,G))."""
        num, den = self._beta_w_partials(xc, xtc, H3c, W3, active, rows=rows)
        num = num.sum(0)
        if den is None:
            den = H3c.sum(dim=2, keepdim=True)              # KL: row sums of H
        else:
            den = den.sum(0)
        return num, den

    def _beta_w_solve(self, blocks, H3, W3, An, Ad, live, iters, block: int = 4):
        """Spectra iterations of one online step (rows ``blocks``; all-reduced under DP).

        Anchored incremental majorisation: every chunk c visited this pass contributes
        An += W_c^(1/gamma) * num_c and Ad += den_c, its MU statistics anchored at the
        spectra W_c it was last stepped from, so W = ((An)/(Ad))^gamma minimises the sum
        of the visited chunks' beta-MU majorisers (for one chunk: exactly sklearn's MU
        step, sklearn/decomposition/_nmf.py:526-728; Lefevre et al. 2011's online IS-NMF
        statistics, generalised to any beta).  The current chunk's term is re-anchored at
        every iteration until |dW|/|W| < ``online_beta_w_tol`` or
        ``online_chunk_max_iter``.  ``An``/``Ad`` hold the OTHER chunks' statistics;
        returns the step's final anchors (an, den) for the caller's bookkeeping."""
        o = self.opts
        kl = self.beta == 1.0
        n, K, G = W3.shape
        X = self.X
        dev, dt = X.device, X.dtype
        g = self._beta_gamma()
        rows = [(a, b) for (a, b) in blocks if b > a]
        hsum = None
        if kl:
            hsum = torch.zeros((n, K), device=dev, dtype=dt)
            for (a, b) in rows:
                hsum += H3[:, :, a:b].sum(dim=2)
            self.comm.allreduce_(hsum)
        an_out = torch.zeros((n, K, G), device=dev, dtype=dt)
        dn_out = None if kl else torch.zeros((n, K, G), device=dev, dtype=dt)
        act = live.clone()
        cuda = dev.type == "cuda"
        dist = self.comm.is_distributed
        sparse = cuda and self._kl_sparse() is not None
        counts = cuda and not sparse and self._kl_counts() is not None
        XT = None if (sparse or counts) else self._xt()
        # the chunk's usages stay fixed over the spectra iterations: split them once
        hpan = {(a, b): self._beta_panels(H3[:, :, a:b]) for (a, b) in rows} \
            if (XT is not None or sparse or counts) else {}
        max_it = int(o.online_chunk_max_iter)
        pending = None
        it = 0
        while it < max_it:
            m = min(block, max_it - it)
            for _ in range(m):
                num = den = None
                for (a, b) in rows:
                    nW, dW = self._beta_w_partials(X[a:b],
                                                   XT[:, a:b] if XT is not None else None,
                                                   H3[:, :, a:b], W3, act, hpan.get((a, b)),
                                                   rows=(a, b))
                    if num is None:
                        num, den = nW, dW
                    else:   # several blocks of one step (single-process DP emulation)
                        num = torch.cat([num, nW])
                        den = torch.cat([den, dW]) if dW is not None else None
                if num is None:    # no local rows (DP rank beyond the data)
                    num = torch.zeros((1, n, K, G), device=dev, dtype=dt)
                    den = None if kl else torch.zeros_like(num)
                if dist:
                    num = num.sum(0, keepdim=True)
                    flat = num.reshape(-1) if kl else torch.cat(
                        [num.reshape(-1), den.sum(0).reshape(-1)])
                    self.comm.allreduce_(flat)
                    num = flat[:n * K * G].view(1, n, K, G)
                    den = None if kl else flat[n * K * G:].view(1, n, K, G)
                ops.beta_w_update(W3, num.contiguous(), None if kl else den.contiguous(), hsum,
                                  An, Ad, an_out, dn_out, self.beta, g, o.l1_W, o.l2_W, o.eps,
                                  o.online_beta_w_tol, act, iters)
            it += m
            if not cuda:
                if int(act.sum()) == 0:
                    break
                continue
            flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
            flag.copy_(act.max().view(1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            prev, pending = pending, (ev, flag)
            if prev is not None:
                prev[0].synchronize()
                if int(prev[1][0]) == 0:
                    break
        # the step's final anchors (replicates that were live at its start)
        return an_out, (hsum if kl else dn_out)

    def _loss_dev(self, HT: torch.Tensor, W: torch.Tensor, K: int) -> torch.Tensor:
        """sqrt(2 * D_beta(X || H W)) per replicate (beta != 2) as a float64 DEVICE tensor
        (no host round trip; all-reduced under DP)."""
        R = W.shape[0] // K
        N, G = self.X.shape
        csr = self._kl_sparse() if HT.device.type == "cuda" else None
        if csr is not None:
            tot = ops.kl_sparse_loss(csr, HT.view(R, K, N), W.view(R, K, G), self.opts.eps)
        else:
            tot = ops.beta_loss(self.X, HT.view(R, K, N), W.view(R, K, G), self.beta,
                                self.opts.eps)
        tot = tot.to(torch.float64).contiguous()
        self.comm.allreduce_(tot)
        return torch.sqrt(torch.clamp(2.0 * tot, min=0.0))

    def _online_beta(self, st: _Batch) -> None:
        """Online beta-MU (nmf-torch mode='online', beta != 2; the mode the reference CLI
        hard-codes, cnmf.py:765, for every --beta-loss, cnmf.py:1426).  Per step the usages
        of its chunk are iterated to ``online_h_tol`` (_beta_h_solve), then the spectra to
        ``online_beta_w_tol`` against the pass's anchored statistics (_beta_w_solve).  The
        statistics restart every pass, as the Frobenius path's.  The pass loss and the
        (prev - cur) / init < tol stop rule stay on the device; the host reads the active
        flags one pass late through the same speculative pass pipeline."""
        o = self.opts
        K = self._beta_K = st.K
        X = self.X
        N, G = X.shape
        steps = self._steps(N)
        kl = self.beta == 1.0
        self._init_err(st)
        pipe = _PassPipeline(st, late_small=False)
        max_pass = int(o.online_max_pass)
        for p in range(max_pass):
            n = st.n_act
            if n == 0:
                break
            HT, W = st.views()
            W3 = W.view(n, K, G)
            H3 = HT.view(n, K, N)
            # the spectra statistics restart every pass (Mairal et al. 2010's schedule, as
            # the Frobenius 'pass' statistics).  Keeping each chunk's majoriser from its
            # last visit instead (incremental MM) was measured: ~30 % fewer spectra
            # iterations but up to 1.7 % worse final KL than batch MU (3000 x 400, K=6)
            An = torch.zeros((n, K, G), device=X.device, dtype=X.dtype)
            Ad = torch.zeros((n, K) if kl else (n, K, G), device=X.device, dtype=X.dtype)
            live = st.active_mask().clone()
            keep = (live != 0).view(n, 1, 1)
            keep_d = keep.view(n, 1) if kl else keep
            for blocks in steps:
                # W is fixed over this step's usage solves
                wpan = self._beta_panels(W3)
                for (a, b) in blocks:
                    if b <= a:
                        continue
                    act = live.clone()
                    self._beta_h_solve(X[a:b], H3[:, :, a:b], W3, act, st.h_iters[:n], wpan,
                                       rows=(a, b))
                an, dn = self._beta_w_solve(blocks, H3, W3, An, Ad, live, st.w_iters[:n])
                An += torch.where(keep, an, 0.0)
                Ad += torch.where(keep_d, dn, 0.0)
            final = p + 1 == max_pass
            st.set_err(self._loss_dev(HT, W, K), p + 1, o.tol, final)
            if not pipe.after_enqueue():
                break

    def _batch_beta(self, st: _Batch) -> None:
        """Batch beta-MU (sklearn _fit_multiplicative_update order: usages, then spectra);
        the W-side statistics are all-reduced under DP, the loss is checked every
        ``loss_every`` iterations."""
        o, comm = self.opts, self.comm
        K = self._beta_K = st.K
        X = self.X
        N, G = X.shape
        self._init_err(st)
        pipe = _PassPipeline(st, late_small=False)
        for it in range(int(o.batch_max_iter)):
            n = st.n_act
            if n == 0:
                break
            HT, W = st.views()
            W3 = W.view(n, K, G)
            H3 = HT.view(n, K, N)
            # finished replicates may sit in the batch until the next (stale-flag)
            # compaction: the active flags gate both updates and the iteration counts
            live = st.active_mask().clone()
            sparse = X.device.type == "cuda" and self._kl_sparse() is not None
            self._beta_h_update(X, H3, W3, o.l1_H, o.l2_H, act=live, rows=(0, N))
            nW, dW = self._beta_w_stats(X, H3, W3, None if sparse else self._xt(), active=live,
                                        rows=(0, N))
            if comm.is_distributed:
                flat = torch.cat([nW.reshape(-1), dW.expand(n, K, G).reshape(-1)])
                comm.allreduce_(flat)
                nW = flat[:n * K * G].view(n, K, G)
                dW = flat[n * K * G:].view(n, K, G)
            self._mu_apply(W3, nW, dW, o.l1_W, o.l2_W, (live != 0).view(n, 1, 1))
            st.h_iters[:n] += live
            st.w_iters[:n] += live
            if (it + 1) % max(1, int(o.loss_every)) == 0 or it + 1 == int(o.batch_max_iter):
                st.set_err(self._loss_dev(HT, W, K), it + 1, o.tol,
                           final=(it + 1 == int(o.batch_max_iter)))
                if not pipe.after_enqueue():
                    break

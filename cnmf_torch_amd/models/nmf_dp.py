"""NMFBatchSolver: the cell-sharded (DP) fused online step: packed reduce-scatter / all-
gather (split out of models/nmf.py)."""
from __future__ import annotations

import torch

from .. import ops
from .nmf_base import _FUSED_MAX_SLABS
from .nmf_batch import _Batch, _Group

# split a single-K batch into two exchange units (halves of its replicates), so each
# half's reduce-scatter / all-gather runs under the other half's compute.  Off: measured
# on MI355X (emulated 8-rank shard, 1M cells x 2000 genes, K=10, 100 replicates) the
# halves' per-rank compute is 0.074 s per step against 0.043 s for one unit -- twice the
# launches of half the size on a launch-bound step -- more than the 0.014 s of
# collectives an ideal overlap could hide (profiles/r5z_emu8_1m_split.json)
_DP_SPLIT = False


def _dp_units(groups, world: int, split: bool | None = None) -> list:
    """The exchange units of a DP fused step: the batch's K groups (a cNMF K grid), or --
    with ``split`` (default _DP_SPLIT) and a batch of ONE K -- its two halves when each
    keeps at least one replicate per rank.  Units are issued in turn, so each unit's
    collectives overlap the other units' compute (_fused_pass_dp)."""
    split = _DP_SPLIT if split is None else split
    if len(groups) != 1 or not split or groups[0].n < 2 * world:
        return list(groups)
    g = groups[0]
    h = (g.n + 1) // 2
    return [_Group(g.K, g.p0, h, g.r0, g.q0),
            _Group(g.K, g.p0 + h, g.n - h, g.r0 + h * g.K, g.q0 + h * g.K * g.K)]


class _DPMixin:
    """NMFBatchSolver methods: the cell-sharded (DP) fused online step: packed reduce-
    scatter / all-gather."""

    # ------------------------------------------------------------------ DP fused step
    def _fused_bufs_dp(self, st: _Batch, steps) -> dict:
        """Workspaces of the cell-sharded fused step (_fused_pass_dp), per K group of the
        batch (a cNMF K grid is one mixed-K batch).  Each group's replicates are
        partitioned into ``world`` equal position chunks of Rr (the last rank's chunk may
        hold fewer real ones); every exchanged buffer is padded to world * Rr positions so
        each rank's chunk is one contiguous block for reduce-scatter / all-gather."""
        xp = self._planes()
        dev = self.X.device
        cws = [b - a for (a, b), in steps]
        units = _dp_units(st.groups, self.comm.world_size)
        # the numerator slab of the widest unit's GEMM plan (a half's split can be deeper)
        slab = max(ops.gemm_plan(g.n * g.K, cw, xp.Gp, xp.pb)[1] * g.n * g.K * cw
                   for cw in cws for g in units)
        f32 = dict(device=dev, dtype=torch.float32)
        groups = [self._fused_bufs_dp_group(g, steps) for g in units]
        self.dp_slices = (min(f["S_h"] for f in groups), min(f["S_w"] for f in groups))
        self.dp_units = len(units)
        return {"units": units, "groups": groups, "prepped": None,
                "slabN": torch.empty(slab, **f32),
                "lin": torch.zeros(st.n_act, **f32), "quad": torch.zeros(st.n_act, **f32)}

    def _fused_bufs_dp_group(self, g, steps) -> dict:
        comm = self.comm
        xp = self._planes()
        dev = self.X.device
        G = self.X.shape[1]
        K, R, world, me = g.K, g.n, comm.world_size, comm.rank
        Rr = -(-R // world)
        Rp = Rr * world
        own0, own1 = min(R, me * Rr), min(R, (me + 1) * Rr)
        cws = [b - a for (a, b), in steps]
        bk = ops.planes_bk(xp.pb)
        kd_max = max(-(-cw // bk) * bk for cw in cws)
        # cooperative slice counts every rank uses (the partial-Gram exchange needs the
        # same number of slots everywhere): from the widest step of ANY rank, and from
        # the full chunk Rr for the W-solve
        cw_max = comm.allreduce_max_int(max(cws))
        S_h = ops.pipe_slices(cw_max, R, K, dev)
        S_w = ops.pipe_slices(G, Rr, K, dev)
        S_h = comm.allreduce_max_int(S_h or 0)
        S_w = comm.allreduce_max_int(S_w or 0)
        if not S_h or not S_w:
            raise RuntimeError("DP fused step: no pipelined-solve slicing")
        f32 = dict(device=dev, dtype=torch.float32)
        wpl_n = ops.gemm_a_planes(xp.Gp)
        # ONE reduce-scatter per online step and group: rank r's chunk is [dB rows of its
        # replicates | their per-slice partial H^T H], and ONE all-gather: rank r's chunk
        # is [the spectra bf16 planes of its replicates | their W W^T partials | lin |
        # quad] as bytes -- the W-solve writes its outputs straight into that chunk
        n_db, n_hh = Rr * K * G, Rr * S_h * K * K
        pl_b, ww_b = wpl_n * Rr * K * xp.Gp * 2, Rr * S_w * K * K * 4
        n_ag = pl_b + ww_b + 8 * Rr
        rs_own = torch.empty(n_db + n_hh, **f32)
        ag_own = torch.zeros(n_ag, device=dev, dtype=torch.uint8)
        return {
            "K": K, "R": R, "Rr": Rr, "Rp": Rp, "own": (own0, own1), "S_h": S_h, "S_w": S_w,
            "wpl_n": wpl_n,
            "wpl": torch.zeros((3, Rp * K, xp.Gp), device=dev, dtype=torch.int16),
            "hpl": torch.zeros((3, R * K, kd_max), device=dev, dtype=torch.int16),
            "dB": torch.zeros((Rp * K, G), **f32),
            "B_own": torch.empty((Rr * K, G), **f32),
            "A_own": [torch.empty((Rr, K, K), **f32) for _ in range(2)],
            "HHp": torch.zeros((Rp, S_h, K, K), **f32),
            "WWp": torch.zeros((Rp, S_w, K, K), **f32),
            "lin": torch.zeros(Rp, **f32), "quad": torch.zeros(Rp, **f32),
            "rs": torch.empty((world, n_db + n_hh), **f32), "rs_own": rs_own,
            "dB_own": rs_own[:n_db].view(Rr * K, G),
            "HHp_own": rs_own[n_db:].view(Rr, S_h, K, K),
            "ag": torch.empty((world, n_ag), device=dev, dtype=torch.uint8), "ag_own": ag_own,
            "ag_pl": ag_own[:pl_b].view(torch.int16).view(wpl_n, Rr * K, xp.Gp),
            "ag_wwp": ag_own[pl_b:pl_b + ww_b].view(torch.float32).view(Rr, S_w, K, K),
            "ag_lin": ag_own[pl_b + ww_b:pl_b + ww_b + 4 * Rr].view(torch.float32),
            "ag_quad": ag_own[pl_b + ww_b + 4 * Rr:].view(torch.float32),
            "ag_offs": (pl_b, ww_b),
            "wwp_n": 1,
        }

    @staticmethod
    def _dp_pack_rs(fb: dict) -> None:
        """[dB | HHp] of every replicate of a group into its reduce-scatter buffer,
        rank-chunked."""
        world = fb["rs"].shape[0]
        n_db = fb["dB_own"].numel()
        rs = fb["rs"]
        rs[:, :n_db].copy_(fb["dB"].view(world, n_db))
        rs[:, n_db:].copy_(fb["HHp"].view(world, -1))

    @staticmethod
    def _dp_unpack_ag(fb: dict, last: bool) -> None:
        """Every rank's chunk of a group's all-gather into the group's planes, W W^T
        partials and (last step) lin / quad."""
        ag = fb["ag"]
        world, Rr, K = ag.shape[0], fb["Rr"], fb["K"]
        pl_b, ww_b = fb["ag_offs"]
        wpl_n = fb["wpl_n"]
        Gp = fb["wpl"].shape[2]
        src = ag[:, :pl_b].view(torch.int16).view(world, wpl_n, Rr * K, Gp)
        fb["wpl"][:wpl_n].view(wpl_n, world, Rr * K, Gp).copy_(src.transpose(0, 1))
        fb["WWp"].view(world, -1).copy_(ag[:, pl_b:pl_b + ww_b].view(torch.float32))
        if last:
            o = pl_b + ww_b
            fb["lin"].view(world, Rr).copy_(ag[:, o:o + 4 * Rr].view(torch.float32))
            fb["quad"].view(world, Rr).copy_(ag[:, o + 4 * Rr:].view(torch.float32))

    def _fused_pass_dp(self, st: _Batch, steps, fball: dict, final: bool) -> None:
        """One online pass of the fused step on a cell shard (SURVEY.md §2.5c / §2.6 item
        1).  Per online step, and per K group of the batch, every rank runs the numerator
        GEMM and the pipelined H-solve on its cells of the global chunk and the statistics
        GEMM dB = H_loc^T X_loc; then ONE reduce-scatter of the packed [dB | partial H^T H]
        hands each rank the rank-summed statistics of ITS replicate chunk, the rank
        W-solves only those (1/world of the spectra work) straight into its chunk of ONE
        all-gather of [bf16 spectra planes | per-slice W W^T partials | lin | quad] -- two
        collectives per step and group (five before the packing: dB, HHp, WWp and one per
        plane, +2 on the last step), the bytes of one all-reduce of dB, the W-solve no
        longer replicated on every rank (the unfused DP step all-reduces [dB | dA] and
        re-solves every replicate everywhere).  Same updates and stopping rules as the
        single-GPU fused step; rank-summed statistics in RCCL's order."""
        o = self.opts
        xp = self._planes()
        HT, W = st.views()
        active = st.active_mask()
        n = st.n_act
        if fball["prepped"] != st.uid:
            # W is replicated at the start of a run: every rank forms every Gram / plane
            for g, fb in zip(fball["units"], fball["groups"]):
                fb["WWp"].zero_()
                fb["WWp"][:g.n, 0].copy_(ops.gram(g.rep3(W)))
                ops.split_planes(W[g.rows], fb["wpl"][:, :g.n * g.K], col_mul=xp.unit)
                fb["wwp_n"] = 1
            fball["prepped"] = st.uid
        units = list(zip(fball["units"], fball["groups"]))
        last_s = len(steps) - 1
        ag_wait = [None] * len(units)
        for s_, ((a, b),) in enumerate(steps):
            # phase 1, per unit: (previous step's all-gather in) numerator GEMM, H-solve,
            # dB GEMM, reduce-scatter issued -- it runs under the next unit's phase 1
            rs_wait = []
            for u, (g, fb) in enumerate(units):
                if ag_wait[u] is not None:
                    ag_wait[u].wait()
                    self._dp_unpack_ag(fb, False)
                rs_wait.append(self._dp_unit_stats(st, g, fb, fball["slabN"], HT, active,
                                                   a, b))
            # phase 2, per unit: W-solve of the owned replicates, all-gather issued -- it
            # runs under the next unit's W-solve (and the next step's phase 1)
            for u, (g, fb) in enumerate(units):
                rs_wait[u].wait()
                ag_wait[u] = self._dp_unit_wsolve(st, g, fb, W, active, s_, s_ == last_s)
        for u, (g, fb) in enumerate(units):
            ag_wait[u].wait()
            self._dp_unpack_ag(fb, True)
        lin, quad = fball["lin"], fball["quad"]
        for g, fb in units:
            lin[g.pos].copy_(fb["lin"][:g.n])
            quad[g.pos].copy_(fb["quad"][:g.n])
        ops.conv_update(lin, quad, self.x_sq, {k: v[:n] for k, v in st.state.items()},
                        n, -1, o.tol, final=final, gate=st.gate,
                        max_pass=int(o.online_max_pass))

    def _dp_unit_stats(self, st: _Batch, g, fb: dict, slabN, HT, active, a: int, b: int):
        """Phase 1 of one unit's online step (see _fused_pass_dp): numerator GEMM and
        pipelined H-solve on this rank's cells of chunk [a, b), the statistics GEMM dB,
        then the packed reduce-scatter, issued in the background; returns its handle."""
        o = self.opts
        xp = self._planes()
        K, R = fb["K"], fb["R"]
        pos = g.pos
        act_g = active[pos]
        h_it = st.h_iters[pos]
        bk = ops.planes_bk(xp.pb)
        rows = R * K
        wpl, hpl_all = fb["wpl"], fb["hpl"]
        wpl_n = fb["wpl_n"]
        cw = b - a
        ks_n = ops.gemm_planes(None, wpl[:wpl_n, :rows], xp.x[:, a:], rows, cw, xp.Gp,
                               raw_slab=slabN, raw_max=_FUSED_MAX_SLABS)
        kd = -(-cw // bk) * bk
        hpl = hpl_all[:, :, :kd]
        hpl_n = ops.gemm_a_planes(kd)
        if cw > 0:
            numer = slabN.as_strided((R, K, cw), (K * cw, cw, 1), 0)
            ops.solve("mu", g.rep3(HT[:, a:b]), numer, None,
                      max_iter=o.online_chunk_max_iter, tol=o.online_h_tol, eps=o.eps,
                      iters_out=h_it, conv_mode=1, check_every=o.inner_check_every,
                      active=act_g, planes=hpl, planes_n=hpl_n, numer_slabs=ks_n,
                      numer_slab_stride=rows * cw, coop=fb["S_h"],
                      gram_parts=fb["WWp"][:R], gram_parts_n=fb["wwp_n"],
                      gram_parts_out=fb["HHp"][:R], coop_device_gen=True)
            ops.gemm_planes(fb["dB"], hpl[:hpl_n], xp.xt[:, :, a:], rows, self.X.shape[1], kd)
        else:      # no cells of this chunk here: zero contributions
            fb["dB"][:rows].zero_()
            fb["HHp"][:R].zero_()
        self._dp_pack_rs(fb)
        return self.comm.reduce_scatter_async(fb["rs_own"], fb["rs"])

    def _dp_unit_wsolve(self, st: _Batch, g, fb: dict, W, active, s_: int, last: bool):
        """Phase 2 of one unit's online step: W-solve of the replicates this rank owns,
        from the rank-summed statistics the reduce-scatter delivered, straight into its
        chunk of the packed all-gather, issued in the background; returns its handle."""
        o = self.opts
        xp = self._planes()
        G = self.X.shape[1]
        K = fb["K"]
        own0, own1 = fb["own"]
        n_own = own1 - own0
        pos = g.pos
        act_g = active[pos]
        w_it = st.w_iters[pos]
        unit = xp.unit
        W_g = W[g.rows]
        Wown = W_g[own0 * K:own1 * K].view(n_own, K, G) if n_own else None
        A_in, A_out = fb["A_own"][(s_ + 1) % 2], fb["A_own"][s_ % 2]
        wwp = fb["ag_wwp"]
        if n_own:
            lin_o = fb["ag_lin"][:n_own]
            quad_o = fb["ag_quad"][:n_own]
            ops.solve(
                "mu", Wown, fb["dB_own"][:n_own * K].view(n_own, K, G),
                None if s_ == 0 else A_in[:n_own], max_iter=o.online_chunk_max_iter,
                tol=o.online_w_tol, eps=o.eps, lin_out=lin_o if last else None,
                quad_out=quad_o if last else None, iters_out=w_it[own0:own1],
                conv_mode=1, check_every=o.inner_check_every, active=act_g[own0:own1],
                planes=fb["ag_pl"][:, :n_own * K], planes_colmul=unit, planes_n=fb["wpl_n"],
                numer_scale=unit,
                numer_base=None if s_ == 0 else fb["B_own"][:n_own * K].view(n_own, K, G),
                numer_out=None if last else fb["B_own"][:n_own * K].view(n_own, K, G),
                gram_parts=fb["HHp_own"][:n_own], gram_parts_n=fb["S_h"],
                gram_out=None if last else A_out[:n_own],
                gram_parts_out=wwp[:n_own], coop=fb["S_w"], coop_device_gen=True)
        fb["wwp_n"] = fb["S_w"]
        return self.comm.all_gather_into_async(fb["ag"], fb["ag_own"])

    def _dp_gather_w(self, st: _Batch, fball: dict) -> None:
        """End of a DP fused run: every rank's W-solved spectra rows to every rank."""
        _, W = st.views()
        me = self.comm.rank
        for g, fb in zip(fball["units"], fball["groups"]):
            K, R, Rr, Rp = fb["K"], fb["R"], fb["Rr"], fb["Rp"]
            W_g = W[g.rows]
            G = W.shape[1]
            Wp = torch.zeros((Rp * K, G), device=W.device, dtype=W.dtype)
            o0, o1 = me * Rr * K, min(R, (me + 1) * Rr) * K
            if o1 > o0:
                Wp[o0:o1].copy_(W_g[o0:o1])
            self.comm.all_gather_into_(Wp, Wp[me * Rr * K:(me + 1) * Rr * K])
            W_g.copy_(Wp[:R * K])
            it = torch.zeros(Rp, dtype=torch.int32, device=W.device)   # W-solve sweeps
            o0, o1 = me * Rr, min(R, (me + 1) * Rr)
            wi = st.w_iters[g.pos]
            if o1 > o0:
                it[o0:o1].copy_(wi[o0:o1])
            self.comm.all_gather_into_(it, it[me * Rr:(me + 1) * Rr])
            wi[:R].copy_(it[:R])

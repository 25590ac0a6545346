"""NMFBatchSolver: continuous batching (run_stream): fixed live positions per K refilled on
the device (split out of models/nmf.py)."""
from __future__ import annotations

import collections
import time

import numpy as np
import torch

from .. import ops
from .nmf_base import NMFResult, _to_device, init_into
from .nmf_batch import _Batch, _Feed, _PassPipeline


class _StreamMixin:
    """NMFBatchSolver methods: continuous batching (run_stream): fixed live positions per K
    refilled on the device."""

    # ------------------------------------------------------------------ streaming
    def stream_live(self, ks) -> dict:
        """Live batch positions per K of a streaming run over the ranks ``ks``: per K the
        replicates ONE co-resident round of the pipelined usage solve holds at the
        online chunk width (ops.pipe_round_reps -- each K group is its own launch), at
        most that K's count.  K > 16 does not stream by default (its count is returned):
        there the usage solve runs in several launch rounds at 100 replicates and the
        replicates run close to online_max_pass (mean 16.8 of 20 passes at K = 20), so
        the batch's tail is short -- measured (profiles/r5e_*): K = 20 streamed 4,928
        (80 slots) / 5,275 (100) vs 5,742 rep/s as one batch; K = 10: 17,570 streamed vs
        14,071.  (run_stream's ``live`` sets the slots explicitly, any K.)"""
        ks = np.asarray(ks, dtype=np.int64)
        N = self.X.shape[0]
        cw = min(N, max(1, int(self.opts.online_chunk_size)))
        out = {}
        for K, cnt in zip(*np.unique(ks, return_counts=True)):
            if K > 16:
                out[int(K)] = int(cnt)
                continue
            m = ops.pipe_round_reps(cw, int(K), self.X.device)
            out[int(K)] = int(min(cnt, m)) if m > 0 else int(cnt)
        return out

    def _stream_ok(self, ks) -> bool:
        o = self.opts
        return (self.X.device.type == "cuda" and self.X.dtype == torch.float32
                and self.beta == 2.0 and o.mode == "online" and o.algo == "mu"
                and o.online_stats == "pass" and o.online_inner_conv == "loss"
                and o.init == "random" and not self.comm.is_distributed
                and all(v == 0.0 for v in (o.l1_H, o.l2_H, o.l1_W, o.l2_W))
                and int(np.max(ks)) <= 32 and not ops.eager_active())

    def run_stream(self, seeds, ks=None, live=None, keep_usages: bool = True,
                   on_result=None) -> NMFResult:
        """Factorise one replicate per seed with CONTINUOUS batching: the batch holds a
        fixed number of live positions per K (``live``: an int for every K or a {K: n}
        dict; default :meth:`stream_live`), and every position whose replicate stopped is
        handed the next staged replicate of the same K at the end of that very pass, on
        the device (stream.hip, inside the pass's captured graph): the finished replicate
        goes to the result store, the staged one -- initialised ahead by the host in a few
        large launches (Philox factors, initial error, W W^T and spectra planes) -- takes
        its position.  Every replicate runs exactly its own solve: its own pass count (the
        device applies ``online_max_pass`` per replicate), convergence rule and
        statistics; only WHICH replicates share a pass changes, so the tail of a ledger
        batch (a few slow replicates the GPU would run alone) overlaps the next
        replicates' passes (the reference runs replicates serially,
        cnmf.py:882-892).  Results are in the callers' order as from :meth:`run`;
        ``keep_usages`` False drops HT (factorize discards usages, cnmf.py:889-892).
        ``on_result`` is called once at the end with (ids, ks, pinned spectra, event) for
        every replicate.  Shapes the streaming path does not take (CPU, beta != 2, HALS,
        DP, K > 32, ...) and requests no larger than the live slots run :meth:`run`."""
        o = self.opts
        seeds = [int(s_) for s_ in seeds]
        R = len(seeds)
        ks = np.full(R, int(o.n_components), dtype=np.int64) if ks is None else \
            np.asarray([int(k) for k in ks], dtype=np.int64)
        if ks.size != R:
            raise ValueError(f"{R} seeds but {ks.size} ranks")
        if R == 0 or not self._stream_ok(ks):
            return self.run(seeds, ks=ks, on_retire=on_result)
        if live is None:
            slots = self.stream_live(ks)
        elif isinstance(live, dict):
            slots = {int(k): int(v) for k, v in live.items()}
        else:
            slots = {int(K): int(live) for K in np.unique(ks)}
        cnt = dict(zip(*[a.tolist() for a in np.unique(ks, return_counts=True)]))
        slots = {K: max(1, min(int(cnt[K]), int(slots.get(K, cnt[K])))) for K in cnt}
        if all(slots[K] >= cnt[K] for K in cnt):
            return self.run(seeds, ks=ks, on_retire=on_result)
        t0 = time.perf_counter()
        N, G = self.X.shape
        dev = self.X.device
        # the feed's device buffers persist per (arena, feed shape): a later run of the same
        # shape (the next ledger batch) replays the passes captured by this one
        kpos_all = np.sort(ks)
        arena = self._arena(np.concatenate([np.repeat(K, slots[K]) for K in sorted(slots)]))
        fkey = (R, tuple(ks.tolist()), bool(keep_usages), tuple(sorted(slots.items())))
        feeds = arena.setdefault("feeds", collections.OrderedDict())
        bufs = feeds.get(fkey)
        if bufs is None:
            bufs = feeds[fkey] = {}
            while len(feeds) > 4:
                feeds.popitem(last=False)
        else:
            feeds.move_to_end(fkey)
        feed = _Feed(seeds, ks, dev, N, G, keep_usages, self.X.dtype, bufs=bufs)
        del kpos_all
        first = []
        for K in sorted(slots):
            q = feed.queue[K]
            first += [q.popleft() for _ in range(slots[K])]
        first = np.asarray(first, dtype=np.int64)
        kpos = ks[first]
        if self._xp is False:
            cw = min(N, int(o.online_chunk_size))
            rows = int(kpos.sum())
            self._ws_reserve = rows * (4 * 4 * (cw + G) + 4 * G + 6 * (cw + G))
        # the stream's batch always lives in an arena (packed state rows the swap kernel
        # reads and writes; the same arena as the feed's above); graphs follow the usual
        # rule
        assert arena is self._arena(kpos)
        HT, W = arena["HT"], arena["W"]
        r0 = 0
        for K in sorted(slots):
            sel = first[kpos == K]
            rws = slice(r0, r0 + sel.size * K)
            init_into(HT[rws], W[rws], self.X, K, [seeds[i] for i in sel], o.init, self.comm,
                      self.row_offset, mean=self._mean(), row_map=self.row_map)
            r0 = rws.stop
        st = _Batch(HT, W, kpos, arena=arena)
        st.graphs = self._graphs_wanted(kpos)
        st.order = first.copy()
        if not self._fused_ok(st, self._steps(N)):
            return self.run(seeds, ks=ks, on_retire=on_result)
        if "ctr" in bufs:          # persistent counters / tables, reset for this run
            feed.ctr, feed.seq, feed.box = bufs["ctr"], bufs["seq"], bufs["box"]
            feed.ctr.zero_()
            feed.seq.zero_()
            feed.box.host.fill_(-1)
        else:
            feed.ctr = bufs["ctr"] = torch.zeros(1 + len(st.groups), dtype=torch.int32, device=dev)
            feed.seq = bufs["seq"] = torch.zeros(1, dtype=torch.int32, device=dev)
            feed.box = bufs["box"] = ops.HostMailbox(1 + len(st.groups))
        for gi, g in enumerate(st.groups):      # rings of an earlier run: heads re-pointed
            if g.K in feed.rings:
                feed.rings[g.K]["head"] = feed.ctr[1 + gi:2 + gi]
        occ_b, plan_b = bufs.setdefault("occ", {}), bufs.setdefault("plan", {})
        for i, g in enumerate(st.groups):
            occ = torch.from_numpy(first[g.p0:g.p0 + g.n].astype(np.int32))
            if g.K in occ_b:
                occ_b[g.K].copy_(occ)
            else:
                occ_b[g.K] = occ.to(dev)
                plan_b[g.K] = torch.empty(2 * g.n, dtype=torch.int32, device=dev)
            feed.occ[g.K] = occ_b[g.K]
            feed.plan[g.K] = plan_b[g.K]
            feed.known_head[g.K] = 0
        st.feed = feed
        self._online_frob(st)
        store = feed.store
        cflags = ops.coop_flags(dev)
        flat = torch.cat([store["sf"][2], store["si"][1:].to(torch.float64).reshape(-1)] +
                         [f.view(-1)[:1].to(torch.float64) for _, f in cflags]).cpu().numpy()
        err, rest = flat[:R], flat[R:5 * R].reshape(4, R)
        if cflags:
            ops.coop_check(values=flat[5 * R:], flags=cflags)
        if on_result is not None:
            host = torch.empty(tuple(store["W"].shape), dtype=store["W"].dtype, pin_memory=True)
            host.copy_(store["W"], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            on_result(np.arange(R), ks.copy(), host, ev)
        stats = {"wall_s": time.perf_counter() - t0,
                 "h_inner_iters": rest[2].astype(np.int64).tolist(),
                 "w_inner_iters": rest[3].astype(np.int64).tolist(),
                 "stream_slots": slots, "stream_stagings": feed.stagings,
                 "stream_passes": feed.passes, "stream_host_wait_s": round(feed.t_wait, 4),
                 "stream_host_stage_s": round(feed.t_stage, 4),
                 "stream_mailbox_misses": feed.box_misses}
        uni = np.unique(ks)
        # (the store is the next run's: hand out copies)
        HTo = store["HT"].clone() if store["HT"] is not None else torch.empty((0, N), device=dev)
        return NMFResult(HT=HTo, W=store["W"].clone(), err=err, n_iter=rest[1].astype(np.int64),
                         converged=rest[0] != 0, seeds=seeds,
                         K=int(uni[0]) if uni.size == 1 else None, stats=stats, ks=ks)

    def _stream_loop(self, st: _Batch, steps, cur: dict) -> None:
        """Pass loop of a streaming run (run_stream).  Each host iteration keeps every
        ring stocked, enqueues one fused pass -- whose end harvests and refills positions
        on the device (_stream_swap_dev) -- and a copy of the counter block, then reads the
        PREVIOUS pass's counters (the GPU never drains): how many replicates were
        harvested (stop at all of them) and how far each ring was consumed (staging room).
        Once nothing waits, positions that emptied are compacted away as in the batch
        pipeline."""
        feed = st.feed
        frac = _PassPipeline(st)._frac
        pending = collections.deque()
        dev = st.W.device
        fb = self._stream_fb(st, cur)
        for g in st.groups:            # every ring exists (and is stocked) before any capture
            self._stream_ring(st, g.K, fb)
            self._stream_stock(st, g.K, cur)
        while True:
            self._enqueue_fused(st, steps, cur)      # ends with the mailbox publish
            ev = torch.cuda.Event()
            ev.record()
            pending.append((ev, feed.passes, st.layout_version))
            feed.passes += 1
            if len(pending) < 2:
                continue
            qev, q, qlv = pending.popleft()
            t_ = time.perf_counter()
            qev.synchronize()
            feed.t_wait += time.perf_counter() - t_
            c = feed.box.read(q)
            if c is None:                           # (never expected) fall back to a copy
                feed.box_misses += 1
                c = feed.ctr.tolist()
            feed.done = c[0]
            if feed.done >= feed.R:
                break
            if qlv != st.layout_version:
                continue
            for i, g in enumerate(st.groups):
                feed.known_head[g.K] = c[1 + i]
            t_ = time.perf_counter()
            for g in st.groups:
                self._stream_stock(st, g.K, cur)
            feed.t_stage += time.perf_counter() - t_
            # drain: nothing waits and every ring is consumed -> a position that emptied
            # stays empty; compact them away (the occupant tables are read back here)
            if feed.waiting() == 0 and all(feed.known_head[g.K] >= feed.rings[g.K]["published"]
                                           for g in st.groups):
                n = st.n_act
                occ_dev = torch.cat([feed.occ[g.K][:g.n] for g in st.groups])
                live = occ_dev.cpu().numpy() >= 0     # (a -1 here is final: nothing to place)
                if not live.any():       # every replicate harvested (done is one pass late)
                    break
                if n - st.prefix_len(live) >= max(1, int(frac(n) * n)):
                    perm = st.compact(live)
                    if perm is not None:
                        self._stream_relayout(st, perm, occ_dev)
                        pending.clear()
        torch.cuda.current_stream(dev).synchronize()

    def _stream_relayout(self, st: _Batch, perm: np.ndarray, occ_dev: torch.Tensor) -> None:
        """After a drain compaction: the occupant tables follow the position permutation
        (st.groups is the new layout), gathered on the DEVICE in stream order -- the pass
        still in flight may harvest more positions after the host read its copy."""
        feed = st.feed
        dev = st.W.device
        occ_new = occ_dev.index_select(0, _to_device(perm[:st.n_act], dev))
        # in place, in the persistent counter block and occupant tables: the new layout's
        # pass graph (captured now or by an earlier run) holds their addresses
        heads = torch.tensor([feed.rings[g.K]["published"] for g in st.groups],
                             dtype=torch.int32)
        feed.ctr[1:1 + len(st.groups)].copy_(heads)
        for gi, g in enumerate(st.groups):
            feed.occ[g.K][:g.n].copy_(occ_new[g.p0:g.p0 + g.n])
            ring = feed.rings[g.K]
            ring["head"] = feed.ctr[1 + gi:2 + gi]

    def _stream_ring(self, st: _Batch, K: int, fb: dict) -> dict:
        """The staging ring of K group: 2 x its live positions of initialised replicates
        (factors, state, W W^T partial-Gram block, spectra planes) at fixed device
        addresses the swap kernel copies from; head (consumed, device, in the feed's
        counter block) / tail (published, device) counters."""
        feed = st.feed
        ring = feed.rings.get(K)
        if ring is not None:
            return ring
        (g,) = [g_ for g_ in st.groups if g_.K == K]
        gi = st.groups.index(g)
        dev = st.W.device
        N, G = self.X.shape
        xp = self._planes()
        S = fb["parts"][g.p0](fb["WWp"]).shape[1]
        qc = 2 * g.n
        ring = {"qc": qc, "block": g.n, "published": 0,
                "head": feed.ctr[1 + gi:2 + gi],
                "tail": torch.zeros(1, dtype=torch.int32, device=dev),
                "ids": torch.full((qc,), -1, dtype=torch.int32, device=dev),
                "W": torch.zeros((qc * K, G), device=dev, dtype=self.X.dtype),
                "HT": torch.zeros((qc * K, N), device=dev, dtype=self.X.dtype),
                "sf": torch.zeros((3, qc), dtype=torch.float64, device=dev),
                "si": torch.zeros((5, qc), dtype=torch.int32, device=dev),
                "parts": torch.zeros((qc, S, K, K), device=dev, dtype=torch.float32),
                "wpl": torch.zeros((3, qc * K, fb["wpl"].shape[2]), device=dev,
                                   dtype=torch.int16)}
        assert fb["wpl"].shape[2] == xp.Gp
        feed.rings[K] = ring
        return ring

    def _stream_stock(self, st: _Batch, K: int, cur: dict) -> None:
        """Stage the next block of waiting replicates of rank K into its ring when the
        ring has a block of room (by the consumed count the host last read): Philox
        factors, their initial error (the init-mode convergence step on the statistics
        _init_err_frob forms), W W^T as partial-Gram slot 0 and the spectra's bf16
        planes, written into the ring slots; then the published count is raised, in
        stream order behind them."""
        feed = st.feed
        qu = feed.queue.get(K)
        if not qu:
            return
        fb = cur["fb"] if cur.get("fb") is not None else self._stream_fb(st, cur)
        ring = self._stream_ring(st, K, fb)
        qc, pub = ring["qc"], ring["published"]
        room = qc - (pub - feed.known_head[K])
        if room < ring["block"]:
            return
        m = min(len(qu), ring["block"])
        o = self.opts
        dev = st.W.device
        N, G = self.X.shape
        xp = self._planes()
        ids = np.asarray([qu.popleft() for _ in range(m)], dtype=np.int64)
        # every staging but the last is a whole block and the ring holds two: a block
        # always starts at slot 0 or `block`, so the replicates are initialised straight
        # into their ring slots (no copies)
        a0 = pub % qc
        assert a0 + m <= qc, "stream ring: staging across the wrap"
        HT_s = ring["HT"][a0 * K:(a0 + m) * K]
        W_s = ring["W"][a0 * K:(a0 + m) * K]
        init_into(HT_s, W_s, self.X, K, feed.seeds[ids].tolist(), o.init, self.comm,
                  self.row_offset, mean=self._mean(), row_map=self.row_map)
        B_s = torch.empty((m * K, G), device=dev, dtype=self.X.dtype)
        self.stats_gemm(B_s, HT_s, 0, N, accumulate=False)
        W3 = W_s.view(m, K, G)
        WW = ops.gram(W3)
        lin = (B_s.view(m, K, G) * W3).sum(dim=(1, 2)).float()
        quad = (ops.gram(HT_s.view(m, K, N)) * WW).sum(dim=(1, 2)).float()
        del B_s
        sf, si = ring["sf"][:, a0:a0 + m], ring["si"][:, a0:a0 + m]
        si.zero_()
        stt = {"err_init": sf[0], "err_prev": sf[1], "err": sf[2], "active": si[0],
               "converged": si[1], "n_pass": si[2]}
        ops.conv_update(lin, quad, self.x_sq, stt, m, 0, o.tol, False, init=True)
        parts = ring["parts"][a0:a0 + m]
        parts.zero_()
        parts[:, 0] = WW
        ops.split_planes(W_s, ring["wpl"][:, a0 * K:(a0 + m) * K], col_mul=xp.unit)
        ring["ids"][a0:a0 + m].copy_(_to_device(ids, dev).to(torch.int32))
        ring["published"] = pub + m
        ring["tail"].fill_(pub + m)
        feed.stagings += 1

    def _stream_fb(self, st: _Batch, cur: dict) -> dict:
        """The fused workspaces of the stream's current layout before its first pass."""
        key = (st.uid, st.layout_version)
        if cur.get("key") != key:
            sl = cur["sl"] = self._slot(st, self._steps(self.X.shape[0])) if st.graphs else None
            cur["fb"] = sl["fb"] if sl is not None else self._fused_bufs(st, self._steps(self.X.shape[0]))
            cur["key"] = key
            cur["fresh"] = True
        return cur["fb"]

    def _stream_swap_dev(self, st: _Batch, fb: dict) -> None:
        """End of a streaming pass: per K group, harvest the stopped replicates and place
        staged ones (ops.stream_swap, stream.hip) -- part of the captured pass."""
        feed = st.feed
        HT, W = st.views()
        sf, si = st.arena["sf"], st.arena["si"]
        store = dict(feed.store)
        store["done"] = feed.ctr[:1]
        for g in st.groups:
            ring = feed.rings.get(g.K)
            if ring is None:
                ring = self._stream_ring(st, g.K, fb)
            grp = {"n": g.n, "K": g.K, "active": st.state["active"][g.pos],
                   "occ": feed.occ[g.K], "plan": feed.plan[g.K],
                   "W": W[g.rows], "HT": HT[g.rows],
                   "parts": fb["parts"][g.p0](fb["WWp"]), "wpl": fb["wpl"][:, g.rows]}
            ops.stream_swap(grp, ring, store, (sf[:, g.p0:], si[:, g.p0:]), st.gate)
        ops.stream_publish(feed.ctr, feed.seq, feed.box)

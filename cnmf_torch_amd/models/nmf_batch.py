"""Replicate-batch state of the NMF engine: the ragged mixed-K batch (_Batch, _Group),
the pass pipeline and the streaming feed (split out of models/nmf.py)."""
from __future__ import annotations

import collections
import itertools
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import ops
from .nmf_base import _to_device



_BATCH_UIDS = itertools.count()



def _ranges(starts: np.ndarray, sizes: np.ndarray) -> np.ndarray:
    """Concatenation of ``arange(s, s + n)`` over the (start, size) pairs."""
    starts = np.asarray(starts, dtype=np.int64)
    sizes = np.asarray(sizes, dtype=np.int64)
    tot = int(sizes.sum())
    if tot == 0:
        return np.zeros(0, dtype=np.int64)
    first = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    return np.repeat(starts - first, sizes) + np.arange(tot, dtype=np.int64)



@dataclass(frozen=True)
class _Group:
    """A run of live positions sharing one K: positions [p0, p0 + n), rows
    [r0, r0 + n*K) of HT / W and K*K-blocks [q0, q0 + n*K*K) of the flat Gram buffers."""

    K: int
    p0: int
    n: int
    r0: int
    q0: int

    @property
    def pos(self) -> slice:
        return slice(self.p0, self.p0 + self.n)

    @property
    def rows(self) -> slice:
        return slice(self.r0, self.r0 + self.n * self.K)

    @property
    def sq(self) -> slice:
        return slice(self.q0, self.q0 + self.n * self.K * self.K)

    def rep3(self, t: torch.Tensor) -> torch.Tensor:
        """(n, K, cols) view of this group's rows of a (rows, cols) tensor or view.  One
        as_strided (no slice + unflatten): ~12 of these per pass sit on the host's enqueue
        path, which is what bounds the few-replicate tail passes."""
        end = self.r0 + self.n * self.K
        if end > t.shape[0]:
            raise IndexError(f"group rows [{self.r0}, {end}) beyond {t.shape[0]}")
        s0, s1 = t.stride()
        return t.as_strided((self.n, self.K, t.shape[1]), (self.K * s0, s0, s1),
                            t.storage_offset() + self.r0 * s0)

    def gram3(self, flat: torch.Tensor) -> torch.Tensor:
        """(n, K, K) view of this group's block of a flat per-position K*K buffer."""
        if self.q0 + self.n * self.K * self.K > flat.shape[0]:
            raise IndexError("group Gram block beyond the buffer")
        K = self.K
        return flat.as_strided((self.n, K, K), (K * K, K, 1), flat.storage_offset() + self.q0)



class _Batch:
    """Live replicate batch with an active-prefix, K-grouped (ragged) layout.

    Replicate position p has rank ``kpos[p]`` and owns ``kpos[p]`` consecutive rows of
    HT (usages transposed) and W (spectra).  Live replicates occupy positions [0, n_act),
    sorted by K, so the live rows of EVERY K form one contiguous prefix: the data-side
    GEMMs of a chunk are single launches over the whole K x n_iter replicate grid while
    the per-replicate solves/Grams run once per K group (``groups``).  ``compact``
    moves finished replicates behind the live ones (``order`` maps position -> original
    replicate id).  Convergence state lives on the device (``state``: float64
    err_init/err_prev/err, int32 active/converged/n_pass) so the solves skip finished
    replicates without a host round trip."""

    def __init__(self, HT, W, kpos, arena: dict | None = None):
        self.HT, self.W = HT, W
        self.kpos = np.asarray(kpos, dtype=np.int64)
        if np.any(np.diff(self.kpos) < 0):
            raise ValueError("replicate positions must be sorted by K")
        R = self.R = int(self.kpos.size)
        self.order = np.arange(R, dtype=np.int64)
        self.n_act = R
        dev = W.device
        # arena (NMFBatchSolver._arena): HT, W and the per-replicate state live in tensors
        # that persist across runs and are compacted IN PLACE, so every buffer a pass
        # touches has the same address for the same layout in every run -- the condition
        # for replaying one captured HIP graph per layout across ledger batches
        self.inplace = arena is not None
        self.arena = arena
        self.graphs = False       # NMFBatchSolver.run: replay graphs per layout (arena only)
        # host-mapped flags slot the last enqueued fused pass stores into (ops.conv_update
        # host_flags), else None: _PassPipeline copies the flags
        self.host_flags = None
        if arena is not None:
            # the arena's per-replicate state is two packed buffers (float64 rows
            # err_init/err_prev/err, int32 rows active/converged/n_pass/h_iters/w_iters):
            # a reset or an in-place compaction is one launch per buffer, not one per field
            self.state = arena["state"]
            arena["sf"].zero_()
            arena["si"].zero_()
            self.h_iters, self.w_iters = arena["h_iters"], arena["w_iters"]
            self.gate = arena["gate"]
        else:
            self.state = {k: torch.zeros(R, dtype=torch.float64, device=dev)
                          for k in ("err_init", "err_prev", "err")}
            for k in ("active", "converged", "n_pass"):
                self.state[k] = torch.zeros(R, dtype=torch.int32, device=dev)
            self.h_iters = torch.zeros(R, dtype=torch.int32, device=dev)
            self.w_iters = torch.zeros(R, dtype=torch.int32, device=dev)
            self.gate = torch.ones(1, dtype=torch.int32, device=dev)
        # device flag "some replicate still active", written by every conv_update: the
        # split GEMMs of the speculative pass enqueued after the batch finished return at
        # once (ops.gemm_planes gate) instead of re-running the last tail pass's products
        self.layout_version = 0   # bumped by compact(): captured graphs key on it
        # optional callback(orig_idx, kpos, host_rows, event): the final spectra of the
        # replicates a compaction retires, copied to pinned memory (ready at `event`), so
        # the caller can persist them while the rest of the batch is still solving
        self.on_retire = None
        self.uid = next(_BATCH_UIDS)   # never reused (unlike id()): plane-cache keys
        # compacted layouts are rounded to this many positions (fewer distinct graphs)
        self.bucket = 8 if W.device.type == "cuda" else 1
        self.A = None   # flat per-position K*K sufficient statistics (online 'exact' mode)
        self.B = None   # (rows, G)
        self.feed = None          # _Feed of a streaming run (NMFBatchSolver.run_stream)
        self._layout()

    def _layout(self) -> None:
        groups = []
        p = r = q = 0
        while p < self.n_act:
            K = int(self.kpos[p])
            e = p
            while e < self.n_act and self.kpos[e] == K:
                e += 1
            groups.append(_Group(K, p, e - p, r, q))
            r += (e - p) * K
            q += (e - p) * K * K
            p = e
        self.groups = groups
        self.rows_act = r
        self.sq_act = q

    @property
    def K(self) -> int:
        """The common K of a single-K batch (the beta != 2 paths need one)."""
        ks = np.unique(self.kpos)
        if ks.size != 1:
            raise ValueError(f"mixed-K batch (K in {ks.tolist()}) has no single K")
        return int(ks[0])

    @property
    def uniform(self) -> bool:
        return np.unique(self.kpos).size == 1

    def views(self):
        return self.HT[:self.rows_act], self.W[:self.rows_act]

    def active_mask(self) -> torch.Tensor:
        return self.state["active"][:self.n_act]

    def _plan(self, act: np.ndarray):
        """(positions kept in the prefix per group, positions moved behind) for the
        host active flags ``act`` of the current prefix.  Each group's live prefix is
        rounded up to a multiple of ``bucket`` replicates (padded with finished ones of
        the same K, which every kernel skips): batch shapes then repeat from step to
        step, so per-shape GEMM tuning is reused instead of re-chosen at every
        compaction."""
        keep, rest = [], []
        for g in self.groups:
            idx = np.arange(g.p0, g.p0 + g.n)
            live = idx[act[idx]]
            dead = idx[~act[idx]]
            n_keep = 0 if live.size == 0 else min(g.n, -(-live.size // self.bucket) * self.bucket)
            pad = n_keep - live.size
            keep.append(np.concatenate([live, dead[:pad]]))
            rest.append(dead[pad:])
        return keep, rest

    def prefix_len(self, act_host: np.ndarray) -> int:
        """Live-prefix length ``compact`` would shrink to for these flags."""
        act = np.asarray(act_host[:self.n_act], dtype=bool)
        return int(sum(k.size for k in self._plan(act)[0]))

    def compact(self, act_host: np.ndarray | None = None) -> None:
        """Move still-active replicates to the front and shrink n_act.

        ``act_host`` (bool per position) may be a STALE host copy of the active flags
        (read one pass behind): flags only ever go 1 -> 0, so every position it marks
        inactive really is finished, and positions that finished since stay in the
        prefix with active = 0 (skipped by the solves) until the next compaction.  The
        permutation is then applied in stream order with no host synchronisation."""
        n = self.n_act
        if act_host is None:
            act_host = self.state["active"][:n].cpu().numpy() != 0
        act = np.asarray(act_host[:n], dtype=bool)
        keep, rest = self._plan(act)
        n_new = int(sum(k.size for k in keep))
        if n_new == n:
            return None
        dev = self.W.device
        if self.swap_ok:
            perm = self._compact_swap(act, n_new)
        else:
            perm = self._compact_gather(keep, rest, n)
        self.order = self.order[perm]
        self.kpos = self.kpos[perm]
        self.n_act = n_new
        self.layout_version += 1
        self._layout()
        if self.on_retire is not None and dev.type == "cuda":
            # positions [n_new, n) are the newly finished ones (flags only go 1 -> 0); their
            # spectra are final: every later kernel skips them, and this copy is in stream
            # order after the last one that wrote them
            roff_new = np.concatenate([[0], np.cumsum(self.kpos)])
            ra, rb = int(roff_new[n_new]), int(roff_new[n])
            host = torch.empty((rb - ra, self.W.shape[1]), dtype=self.W.dtype, pin_memory=True)
            host.copy_(self.W[ra:rb], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self.on_retire(self.order[n_new:n].copy(), self.kpos[n_new:n].copy(), host, ev)
        return perm

    @property
    def swap_ok(self) -> bool:
        """Compaction by in-place position swaps (``_compact_swap``): a single-K arena batch
        without per-position statistics (the 'exact' online mode's A / B).  Mixed-K
        batches shift whole groups when one shrinks and keep the gather form."""
        return (self.inplace and len(self.groups) == 1 and self.B is None
                and os.environ.get("CNMF_COMPACT_SWAP", "1") != "0")

    def _compact_swap(self, act: np.ndarray, n_new: int) -> np.ndarray:
        """The live replicates beyond the new prefix [0, n_new) trade places with finished
        ones inside it -- disjoint swaps, one kernel (ops.rows_swap), and only the movers'
        rows are touched.  Positions [n_new, n) then hold finished replicates only, as
        after the gather form (the padding of the bucketed prefix stays finished ones)."""
        n = self.n_act
        K = int(self.kpos[0])
        idx = np.arange(n)
        holes = idx[:n_new][~act[:n_new]]
        movers = idx[n_new:][act[n_new:]]
        m = movers.size
        assert m <= holes.size
        perm = np.arange(self.R, dtype=np.int64)
        perm[holes[:m]] = movers
        perm[movers] = holes[:m]
        if m:
            pairs = np.empty(2 * m, dtype=np.int32)
            pairs[0::2], pairs[1::2] = holes[:m], movers
            pt = torch.from_numpy(pairs)
            if self.W.device.type == "cuda":
                pt = pt.pin_memory().to(self.W.device, non_blocking=True)
            ops.rows_swap(pt, K, [self.HT, self.W], self.arena["sf"], self.arena["si"])
        return perm

    def _compact_gather(self, keep, rest, n: int) -> np.ndarray:
        perm = np.concatenate(keep + rest + [np.arange(n, self.R)]).astype(np.int64)
        dev = self.W.device
        roff = np.concatenate([[0], np.cumsum(self.kpos)[:-1]])
        rows = _to_device(_ranges(roff[perm], self.kpos[perm]), dev)
        pidx = _to_device(perm, dev)
        if self.inplace:     # same storage, permuted rows (arena: addresses never move)
            for t, ix in ((self.HT, rows), (self.W, rows)):
                t.copy_(t.index_select(0, ix))
            for t in (self.arena["sf"], self.arena["si"]):
                t.copy_(t.index_select(1, pidx))
        else:
            self.HT = self.HT.index_select(0, rows)
            self.W = self.W.index_select(0, rows)
            self.state = {k: v.index_select(0, pidx) for k, v in self.state.items()}
            self.h_iters = self.h_iters.index_select(0, pidx)
            self.w_iters = self.w_iters.index_select(0, pidx)
        if self.B is not None:
            self.B = self.B.index_select(0, rows)
            sq = self.kpos * self.kpos
            qoff = np.concatenate([[0], np.cumsum(sq)[:-1]])
            self.A = self.A.index_select(0, _to_device(_ranges(qoff[perm], sq[perm]), dev))
        return perm

    def set_err(self, err: torch.Tensor, pass_idx: int, tol: float, final: bool,
                init: bool = False) -> None:
        """Host-computed per-position errors (beta != 2 paths) -> same bookkeeping as the
        device convergence kernel."""
        n = self.n_act
        st = self.state
        e = err[:n].to(device=st["err"].device, dtype=torch.float64)
        if init:
            for k in ("err_init", "err_prev", "err"):
                st[k][:n] = e
            st["active"][:n] = 1
            return
        act = st["active"][:n] != 0
        st["err"][:n] = torch.where(act, e, st["err"][:n])
        st["n_pass"][:n] = torch.where(act, torch.full_like(st["n_pass"][:n], pass_idx),
                                       st["n_pass"][:n])
        rel = (st["err_prev"][:n] - e) / torch.clamp(st["err_init"][:n], min=1e-300)
        conv = act & (rel < tol)
        stop = conv | (act & bool(final))
        st["converged"][:n] = torch.where(conv, torch.ones_like(st["converged"][:n]),
                                          st["converged"][:n])
        st["err_prev"][:n] = torch.where(act & ~stop, e, st["err_prev"][:n])
        st["active"][:n] = torch.where(stop, torch.zeros_like(st["active"][:n]),
                                       st["active"][:n])

    def finalize(self, extra=()):
        """Restore original replicate order: (HT, W, ks, err, n_pass, converged,
        h_iters, w_iters, extra_values), rows of replicate r at offs[r] : offs[r] + ks[r].
        ``extra``: one-element int device tensors (the cooperative-solve flags) read back
        in the same copy, as a float64 array."""
        inv = np.argsort(self.order)
        dev = self.W.device
        roff = np.concatenate([[0], np.cumsum(self.kpos)[:-1]])
        rows = _to_device(_ranges(roff[inv], self.kpos[inv]), dev)
        HT = self.HT.index_select(0, rows)
        W = self.W.index_select(0, rows)
        # the raw per-position state goes to the host as it lies (an arena batch: its two
        # packed buffers, two copies) and is put in replicate order there -- the device
        # gather / cast / stack of every field cost ~10 small launches at each run's end,
        # host-latency bound (profiles/r6zl_*)
        R = self.R
        if self.arena is not None:
            srcs = [self.arena["sf"], self.arena["si"]]
        else:
            srcs = [self.state["err"], self.state["n_pass"], self.state["converged"],
                    self.h_iters, self.w_iters]
        srcs = srcs + [t.view(-1)[:1] for t in extra]
        if dev.type == "cuda":
            host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in srcs]
            for hb, t in zip(host, srcs):
                hb.copy_(t, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            host = [hb.numpy() for hb in host]
        else:
            host = [t.numpy().copy() for t in srcs]
        if self.arena is not None:
            sf, si = host[0], host[1]
            err, conv, n_pass, hi, wi = sf[2, :R], si[1, :R], si[2, :R], si[3, :R], si[4, :R]
            ext_h = host[2:]
        else:
            err, n_pass, conv, hi, wi = (h[:R] for h in host[:5])
            ext_h = host[5:]
        ext = np.array([float(e.reshape(-1)[0]) for e in ext_h], dtype=np.float64)
        return (HT, W, self.kpos[inv], err[inv].astype(np.float64),
                n_pass[inv].astype(np.int64), conv[inv] != 0, hi[inv].astype(np.int64),
                wi[inv].astype(np.int64), ext)



class _PassPipeline:
    """Host side of the speculative pass loop.

    Pass p is enqueued before the host knows whether pass p-1 finished everybody: the
    active flags of pass p-1 are copied to pinned memory asynchronously and read one pass
    behind, so the GPU never drains at a pass boundary.  When flags show that enough
    replicates finished, the host synchronises once and compacts the batch."""

    def __init__(self, st: _Batch, compact_frac: float | None = None,
                 late_small: bool = True):
        self.st = st
        self.cuda = st.W.device.type == "cuda"
        explicit = compact_frac is not None
        if compact_frac is None:
            compact_frac = float(os.environ.get("CNMF_COMPACT_FRAC", "0.25"))
        self.frac = compact_frac
        # batches of <= 256 replicates compact later: at that size the GEMMs are latency-
        # bound, so dropping finished replicates saves little GPU time while each
        # compaction costs host enqueue time (permutation, re-split of W) -- measured on
        # MI355X (profiles/r2_compact_frac_ab.txt): 100 replicates 10,487 -> 10,956 rep/s
        # at 0.75 vs 0.25; the 900-replicate K grid loses 3.5 % at 0.5, so it keeps 0.25
        # (``late_small`` False: the beta != 2 solvers, GPU-bound at every batch size --
        # their elementwise passes over X shrink with every retired replicate)
        self.frac_small = compact_frac if (explicit or not late_small) else \
            float(os.environ.get("CNMF_COMPACT_FRAC_SMALL", "0.75"))
        # single-K arena batches compact by in-place swaps (_Batch._compact_swap: only the
        # movers' rows, one launch), cheap enough to shrink the batch at every bucket of
        # finished replicates (CNMF_COMPACT_FRAC_SWAP; 0 = any shrink of the prefix)
        self.swap = not explicit and "CNMF_COMPACT_FRAC_SMALL" not in os.environ
        self.frac_swap = float(os.environ.get("CNMF_COMPACT_FRAC_SWAP", "0"))
        self.pending = None   # (event, host_flags, n)

    def _frac(self, n: int) -> float:
        # (the policy depends on the batch's shape only, never on whether it compacts by
        # swaps or gathers: the compacted layouts re-plan the GEMMs' k split, so two runs
        # of the same replicates agree bit for bit only through the same layouts)
        # (a streaming run's drain compactions read its occupant tables back: they keep
        # the late policy)
        if self.swap and self.cuda and len(self.st.groups) == 1 and self.st.feed is None and \
                os.environ.get("CNMF_COMPACT_SWAP", "1") != "0":
            return self.frac_swap
        return self.frac_small if n <= 256 else self.frac

    def after_enqueue(self) -> bool:
        """Call after enqueueing a pass (incl. its convergence update).  Returns False
        when the loop should stop."""
        st = self.st
        n = st.n_act
        if not self.cuda:
            n_live = int((st.state["active"][:n] != 0).sum())
            if n_live == 0:
                return False
            if n - st.prefix_len(st.state["active"][:n].numpy() != 0) >= max(1, int(self._frac(n) * n)):
                st.compact()
            return True
        hf, st.host_flags = st.host_flags, None
        if hf is not None and hf.numel() == n:
            # this pass's flags, stored by its conv_update into a host-mapped slot; the next
            # pass stores into the other slot, so the read below (after this pass's event,
            # one pass later) sees exactly this pass's flags -- no copy launch
            flags = hf
        else:
            flags = torch.empty(n, dtype=torch.int32, pin_memory=True)
            # (a flag copy on a side stream removed the ~5 us gap per pass in the trace but
            # was slower end to end -- headline -2 %, K grid -5.5 %, profiles/r3y_*: the
            # stream switch and event sit on the host's enqueue path)
            flags.copy_(st.state["active"][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        prev, self.pending = self.pending, (ev, flags, n)
        if prev is None:
            return True
        pev, pflags, pn = prev
        pev.synchronize()
        if pn != n:                       # a compaction happened in between: stale layout
            return True
        n_live = int((pflags != 0).sum())
        if n_live == 0:                   # everything had finished one pass ago
            return False
        flags_np = pflags.numpy() != 0
        if n - st.prefix_len(flags_np) >= max(1, int(self._frac(n) * n)):
            # compact on the one-pass-stale flags, in stream order: no drain of the GPU
            st.compact(flags_np)
            self.pending = None
            return st.n_act > 0
        return True



_FEED_UIDS = itertools.count()



class _Feed:
    """State of a streaming run (NMFBatchSolver.run_stream).  Host side: the replicates
    still waiting, one queue per K in ledger order, and per K group a RING of staged
    (initialised) replicates with the count the host has published into it.  Device side:
    the result store every finished replicate is copied into (rows of replicate i at
    ``offs[i]``, as NMFResult), the per-position occupant tables, the rings, and a small
    counter block (harvested count, each ring's consumed count) the host reads one pass
    late (stream.hip: the swap runs inside the pass)."""

    def __init__(self, seeds, ks, dev, N: int, G: int, keep_usages: bool,
                 dtype=torch.float32, bufs: dict | None = None):
        """``bufs`` (a dict the caller keeps per arena and feed shape): the device buffers
        -- result store, rings, counters, occupant tables, mailbox -- persist there across
        runs at fixed addresses, so a pass graph captured by one run replays in the next
        (``buf_uid`` keys the graph slots); they are reset here, and the results handed
        out are copies (the next run reuses the store)."""
        self.uid = next(_FEED_UIDS)
        self.seeds = np.asarray(seeds, dtype=np.int64)
        self.ks = np.asarray(ks, dtype=np.int64)
        R = self.seeds.size
        self.offs = np.concatenate([[0], np.cumsum(self.ks)[:-1]]).astype(np.int64)
        self.queue = {int(K): collections.deque(np.flatnonzero(self.ks == K).tolist())
                      for K in np.unique(self.ks)}
        tot = int(self.ks.sum())
        self.bufs = bufs
        if bufs is not None and "store" in bufs:
            self.store = bufs["store"]
            self.store["sf"].zero_()
            self.store["si"].zero_()
        else:
            self.store = {
                "offs": torch.from_numpy(self.offs).to(dev),
                "W": torch.empty((tot, G), device=dev, dtype=dtype),
                "HT": torch.empty((tot, N), device=dev, dtype=dtype) if keep_usages else None,
                # err_init, err_prev, err | active, converged, n_pass, h_iters, w_iters
                "sf": torch.zeros((3, R), dtype=torch.float64, device=dev),
                "si": torch.zeros((5, R), dtype=torch.int32, device=dev),
            }
            if bufs is not None:
                bufs["store"] = self.store
                bufs["uid"] = next(_FEED_UIDS)
        self.buf_uid = bufs["uid"] if bufs is not None else self.uid
        self.R = R
        # K -> ring (see NMFBatchSolver._stream_ring); persistent rings restart empty
        self.rings: dict = bufs.setdefault("rings", {}) if bufs is not None else {}
        for ring in self.rings.values():
            ring["published"] = 0
            ring["tail"].zero_()
            ring["ids"].fill_(-1)
        self.ctr = None           # int32 device [1 + n_rings]: harvested, ring heads
        self.occ: dict = {}       # K -> int32 device occupant table of the group
        self.plan: dict = {}      # K -> int32 device [2 n] swap plan scratch
        self.known_head: dict = {}
        self.done = 0             # harvested count the host has seen
        self.passes = 0
        self.stagings = 0
        self.t_wait = self.t_stage = 0.0
        self.box_misses = 0       # mailbox rows that did not carry the expected pass

    def waiting(self) -> int:
        return sum(len(q) for q in self.queue.values())

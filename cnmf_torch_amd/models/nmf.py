"""Replicate-batched NMF engine (replaces nmf-torch ``run_nmf``).

The reference factorises one replicate at a time (``cNMF._nmf`` -> ``run_nmf``,
cnmf.py:805-821, serial loop cnmf.py:882-892).  Here a *batch* of R replicates that
share X and K is solved together:

* the data-side products are single fat GEMMs over the whole batch
  (``W_all @ X_c^T`` is (R*K x G)(G x c), ``H_all^T @ X_c`` is (R*K x c)(c x G));
* the per-replicate inner loops (H with W fixed, W with H fixed) are ONE launch of the
  fused solve kernel for every replicate (csrc/kernels/solve.hip), converging on device;
* the Frobenius loss comes for free from sufficient statistics (trace trick) in the
  W-solve epilogue -- no extra pass over X;
* replicates that have converged are compacted out of the batch so later passes only
  pay for live ones; every replicate still runs exactly its own convergence history.

Layouts: ``W`` is (R*K, G) row-major (replicate r = rows r*K..r*K+K-1) and the usages
are kept TRANSPOSED, ``HT`` (R*K, N), so a replicate's chunk block is K rows of
contiguous cells -- coalesced for the solve kernel and directly the GEMM operand.

Algorithms (nmf-torch surface; cnmf.py:757-771 fixes algo='mu', mode='online'):
  algo  in {'mu', 'hals', 'halsvar', 'bpp'} (all but MU: Frobenius only; bpp = exact
                                 NNLS half-steps, models/bpp.py; halsvar = HALS inner loops
                                 run to ``batch_hals_tol`` to mimic bpp's exact half-steps)
  mode  in {'online', 'batch'}
  beta_loss in {'frobenius', 'kullback-leibler', 'itakura-saito'} or a float
Online (Mairal-style sufficient statistics): per pass, chunks of ``online_chunk_size``
rows; H-step on the chunk to ``online_h_tol`` (relative change over the chunk, as
cnmf.py:375-378), accumulate A += h^T h, B += h^T x, then W-step to ``online_w_tol``.
A pass ends with the loss; stop when (prev - cur) / init < tol or after
``online_max_pass`` passes.  Chunks are taken in row order (deterministic and identical
for every replicate of a batch -- required for batching; documented deviation from a
shuffled order).  For beta != 2, the W-step accumulates the MU numerator/denominator
with the current W and applies one multiplicative step per chunk.
Batch: alternate one H-step and one W-step -- one MU / HALS sweep each ('mu', 'hals'),
HALS inner loops to ``batch_hals_tol`` / ``batch_hals_max_iter`` ('halsvar'), or an exact
NNLS solve ('bpp') -- loss every ``loss_every`` iterations, stop as sklearn's MU solver
does.  In online mode 'halsvar' equals 'hals' (the chunk solves already iterate to
``online_h_tol`` / ``online_w_tol``).  nmf-torch is not installed here, so the
hals / halsvar split follows its documented parameter roles (parity unpinned).

Data parallel (cell-sharded) runs pass a communicator: the flat per-chunk ``[dB | dA]``
increment is all-reduced once per online step, so W, the loss and every convergence
decision are identical on all ranks while H rows stay rank-local.

Modules: nmf_base (options, init, X operands), nmf_batch (batch state),
nmf_graphs / nmf_stream / nmf_dp / nmf_beta (NMFBatchSolver mixins).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .. import ops
from ..parallel.comm import LocalComm
from .nmf_base import (  # noqa: F401
    NMFOptions,
    NMFResult,
    PlanesOnlyX,
    _FUSED_MAX_SLABS,
    _LAYOUT_REPLAY,
    _XPlanes,
    _chunks,
    _global_mean,
    _graphs_enabled,
    _inner_solve,
    _sq_norm,
    _to_device,
    _warn_once,
    beta_value,
    init_into,
    kernel_max_rank,
    log,
    native_rank,
)
from .nmf_batch import _Batch, _PassPipeline, _ranges
from .nmf_graphs import _GraphMixin
from .nmf_stream import _StreamMixin
from .nmf_dp import _DPMixin
from .nmf_beta import _BetaMixin

# re-exports: the engine's public and test-facing names live in the split modules
from .nmf_base import *  # noqa: F401,F403,E402
from .nmf_base import (  # noqa: F401,E402
    _FUSED_MAX_SLABS,
    _LAYOUT_REPLAY,
    _SQ_NORM_CACHE,
    _WARNED,
    _XPlanes,
    _block_colstats,
    _chunks,
    _count_units,
    _global_mean,
    _graphs_enabled,
    _inner_solve,
    _nndsvd,
    _sq_norm,
    _to_device,
    _warn_once,
)
from .nmf_batch import (  # noqa: F401,E402
    _BATCH_UIDS,
    _Batch,
    _FEED_UIDS,
    _Feed,
    _Group,
    _PassPipeline,
    _ranges,
)



class NMFBatchSolver(_GraphMixin, _StreamMixin, _DPMixin, _BetaMixin):
    """Solve R replicates (same X, same K, different seeds) together."""

    def __init__(self, X: torch.Tensor, opts: NMFOptions, comm=None, row_offset: int = 0,
                 profile: bool = False, schedule=None, row_map=None):
        opts.validate()
        # optional explicit online schedule: list of steps, each a list of (row_start,
        # row_end) blocks solved independently before one W update (used to emulate the
        # cell-sharded schedule in a single process)
        self.schedule = schedule
        self.opts = opts
        self.comm = comm or LocalComm()
        self._virtual = isinstance(X, PlanesOnlyX)
        if self._virtual:
            # planes only: X stands in as a NaN-valued (N, G) view of one element -- shape,
            # device and dtype for the bookkeeping; any read of its values would surface as
            # NaN errors, and every code path that reads X raises before it
            if beta_value(opts.beta_loss) != 2.0 or \
                    opts.mode != "online" or opts.online_stats != "pass" or \
                    opts.init != "random" or opts.algo not in ("mu", "hals") or \
                    opts.dtype != torch.float32:
                raise ValueError("PlanesOnlyX supports online Frobenius MU/HALS with random "
                                 "init in float32 (the planes are the only copy of X)")
            src = X
            X = torch.full((1, 1), float("nan"), device=src.device).expand(*src.shape)
        self.X = X if X.dtype == opts.dtype else X.to(opts.dtype)
        self.row_offset = row_offset
        # [(local_start, local_stop, global_start)]: where this rank's rows sit in the
        # global matrix (a chunk-interleaved DP shard; see parallel.runner.dp_row_segments)
        self.row_map = row_map
        self.beta = beta_value(opts.beta_loss)
        self.profile = profile
        self.timings: dict[str, float] = {}
        # ||X||_F^2 (global) for the trace-trick loss; on the GPU from the fused column
        # statistics pass that also feeds the split-GEMM count detection
        self._colstats = None
        self._mean_x = None
        self._xp = False            # split-GEMM planes of X: False = not built yet
        self._ws_reserve = 0        # bytes of per-batch workspaces still to allocate (run)
        if self._virtual:
            local_sq = src.x_sq
            self._xp = src.planes
            self._mean_x = self.comm.allreduce_scalar(src.sum) / max(
                self.comm.allreduce_scalar(float(src.shape[0] * src.shape[1])), 1.0)
        elif self.X.device.type == "cuda" and self.X.dtype == torch.float32 and self.X.numel():
            self._colstats = ops.colstats(self.X)
            local_sq = float(self._colstats[1].sum())
        else:
            local_sq = _sq_norm(self.X)
        self.x_sq = self.comm.allreduce_scalar(local_sq)
        self._ws: dict = {}
        self._w_fresh: dict = {}    # stream -> key of the W its "w" planes hold
        self._XT = None             # X^T (G, N padded to 4) for the beta W-side kernel
        self._beta_K = 0            # rank of the beta != 2 batch being solved (padded)

    # ------------------------------------------------------------------ public
    def run(self, seeds, HT0=None, W0=None, ks=None, on_retire=None) -> NMFResult:
        """Factorise one replicate per seed.  ``ks`` (one K per seed; default
        ``opts.n_components`` for all) may mix ranks: the Frobenius solvers then run the
        whole K x n_iter grid as ONE ragged batch (one pass loop, one data-side GEMM per
        chunk for every K).  The beta != 2 solvers take one K at a time; a mixed-K
        request is split by K for them.  ``on_retire`` (GPU, unpadded ranks): called
        with (indices into ``seeds``, their K, pinned spectra rows, event) for the
        replicates each compaction retires -- their final spectra, ready once the event
        completes -- while the remaining ones keep solving (see _Batch.compact)."""
        o = self.opts
        seeds = [int(s_) for s_ in seeds]
        R = len(seeds)
        ks = np.full(R, int(o.n_components), dtype=np.int64) if ks is None else \
            np.asarray([int(k) for k in ks], dtype=np.int64)
        if ks.size != R:
            raise ValueError(f"{R} seeds but {ks.size} ranks")
        if R and ks.min() < 1:
            raise ValueError("every K must be >= 1")
        kmax = kernel_max_rank(self.beta, o.algo)
        uncovered = (self.X.device.type == "cuda" and not ops.eager_active() and R
                     and kmax is not None and int(ks.max()) > kmax)
        if (self.beta != 2.0 or uncovered) and np.unique(ks).size > 1:
            if on_retire is not None:
                raise ValueError("on_retire needs a single K for beta != 2 or K > "
                                 f"{kmax}")
            return self._run_split_by_k(seeds, ks)
        if uncovered:
            # no kernel instantiation for this rank: run the PyTorch reference ops on the
            # same GPU instead of failing the job (logged once per K)
            _warn_once(f"K={int(ks[0])}: the native gfx950 kernels cover K <= {kmax} for "
                       f"beta_loss={self.opts.beta_loss!r}, algo={o.algo!r}; these "
                       "replicates run the eager PyTorch ops on the GPU (slower)")
            log.info("K=%d > %d: eager PyTorch routing on %s", int(ks[0]), kmax, self.X.device)
            with ops.eager_ops():
                return self.run(seeds, HT0=HT0, W0=W0, ks=ks, on_retire=None)
        t0 = time.perf_counter()
        # wide ranks run padded on the GPU kernels (native_rank); bpp solves on torch linalg
        pad = self.X.device.type == "cuda" and o.algo != "bpp" \
            and bool((ks > 32).any()) and not ops.eager_active()
        kp = np.array([native_rank(k) for k in ks], dtype=np.int64) if pad else ks
        pos = np.lexsort((np.arange(R), kp, ks))     # positions grouped by K
        kpos = kp[pos]
        arena = None
        if HT0 is None or W0 is None:
            N, G = self.X.shape
            tot = int(kpos.sum())
            arena = self._arena(kpos) if self._graphs_wanted(kpos) else None
            if arena is not None:
                # init_into overwrites every row of an unpadded block; the zero padding
                # components of a padded one (native_rank) are cleared here
                HT, W = arena["HT"], arena["W"]
                if pad:
                    HT.zero_()
                    W.zero_()
            else:
                HT = torch.zeros((tot, N), device=self.X.device, dtype=self.X.dtype)
                W = torch.zeros((tot, G), device=self.X.device, dtype=self.X.dtype)
            r0 = 0
            for K in np.unique(ks[pos]):
                sel = pos[ks[pos] == K]
                Kp = int(kp[sel[0]])
                rows = slice(r0, r0 + sel.size * Kp)
                if Kp == K:
                    init_into(HT[rows], W[rows], self.X, int(K), [seeds[i] for i in sel],
                              o.init, self.comm, self.row_offset, mean=self._mean(),
                              row_map=self.row_map)
                else:   # rank-K init in the first K rows of each padded block
                    h_ = torch.empty((sel.size * int(K), N), device=HT.device, dtype=HT.dtype)
                    w_ = torch.empty((sel.size * int(K), G), device=W.device, dtype=W.dtype)
                    init_into(h_, w_, self.X, int(K), [seeds[i] for i in sel], o.init,
                              self.comm, self.row_offset, mean=self._mean(),
                              row_map=self.row_map)
                    HT[rows].view(sel.size, Kp, N)[:, :K] = h_.view(sel.size, K, N)
                    W[rows].view(sel.size, Kp, G)[:, :K] = w_.view(sel.size, K, G)
                r0 = rows.stop
        else:
            if np.unique(ks).size > 1:
                raise ValueError("explicit initial factors need a single K")
            if pad:
                raise ValueError("explicit initial factors need K <= 32 on the GPU")
            HT, W = HT0.to(self.X.dtype).clone(), W0.to(self.X.dtype).clone()
        if self._xp is False:
            # the fused step's workspaces for this batch, allocated after the X planes:
            # <= 4 raw split-K slabs of both GEMMs, the accumulated B, 3 bf16 planes of
            # the usages and spectra (a generous bound; _fused_bufs)
            N, G = self.X.shape
            rows = int(kpos.sum())
            cw = min(N, int(o.online_chunk_size))
            self._ws_reserve = rows * (4 * 4 * (cw + G) + 4 * G + 6 * (cw + G))
        st = _Batch(HT, W, kpos, arena=arena)
        st.graphs = arena is not None
        st.order = pos.astype(np.int64).copy()
        if on_retire is not None and not pad:
            st.on_retire = on_retire
        if self.beta == 2.0:
            if o.mode == "online":
                self._online_frob(st)
            else:
                self._batch_frob(st)
        else:
            if o.mode == "online":
                self._online_beta(st)
            else:
                self._batch_beta(st)
        # the cooperative solves' failure flags ride in finalize's one device->host copy
        cflags = ops.coop_flags(self.X.device) if self.X.device.type == "cuda" else []
        HT, W, ks_out, err, n_iter, conv, hi, wi, cvals = st.finalize([f for _, f in cflags])
        if pad:     # drop the zero padding components: rows [0, K) of each block
            offp = np.concatenate([[0], np.cumsum(ks_out)[:-1]])
            keep = _to_device(_ranges(offp, ks), HT.device)
            HT, W = HT.index_select(0, keep), W.index_select(0, keep)
            ks_out = ks
        if cflags:
            ops.coop_check(values=cvals, flags=cflags)
        check = getattr(self.comm, "check", None)
        if check is not None:     # one-shot xGMI all-reduce gave up on a peer?  Raise
            check()               # before any caller can persist these spectra
        stats = {"wall_s": time.perf_counter() - t0, "h_inner_iters": hi.tolist(),
                 "w_inner_iters": wi.tolist()}
        uni = np.unique(ks_out)
        return NMFResult(HT=HT, W=W, err=err, n_iter=n_iter, converged=conv, seeds=seeds,
                         K=int(uni[0]) if uni.size == 1 else None, stats=stats, ks=ks_out)

    def _run_split_by_k(self, seeds, ks) -> NMFResult:
        """One single-K run per distinct K, merged back into the callers' order."""
        t0 = time.perf_counter()
        parts = {}
        for K in np.unique(ks):
            idx = np.flatnonzero(ks == K)
            parts[int(K)] = (idx, self.run([seeds[i] for i in idx], ks=[int(K)] * idx.size))
        R = len(seeds)
        err, n_iter = np.zeros(R), np.zeros(R, dtype=np.int64)
        conv = np.zeros(R, dtype=bool)
        hi, wi = [0] * R, [0] * R
        offs = np.concatenate([[0], np.cumsum(ks)[:-1]])
        dev = self.X.device
        HT = torch.empty((int(ks.sum()), self.X.shape[0]), device=dev, dtype=self.X.dtype)
        W = torch.empty((int(ks.sum()), self.X.shape[1]), device=dev, dtype=self.X.dtype)
        for K, (idx, res) in parts.items():
            rows = _to_device(_ranges(offs[idx], ks[idx]), dev)
            HT.index_copy_(0, rows, res.HT)
            W.index_copy_(0, rows, res.W)
            err[idx], n_iter[idx], conv[idx] = res.err, res.n_iter, res.converged
            for j, i in enumerate(idx):
                hi[i] = res.stats["h_inner_iters"][j]
                wi[i] = res.stats["w_inner_iters"][j]
        stats = {"wall_s": time.perf_counter() - t0, "h_inner_iters": hi, "w_inner_iters": wi}
        return NMFResult(HT=HT, W=W, err=err, n_iter=n_iter, converged=conv, seeds=list(seeds),
                         K=None, stats=stats, ks=ks)

    # ------------------------------------------------------------------ data-side GEMMs
    def _planes(self):
        """X planes for the split-precision MFMA GEMMs, or None (CPU, fp64, memory)."""
        if self._xp is False:
            self._xp = _XPlanes.build(self.X, self._colstats, reserve=self._ws_reserve)
        return self._xp

    def _plane_buf(self, key: str, rows: int, cols: int) -> torch.Tensor:
        """(3, rows, cols) int16 workspace, reused while the shape holds."""
        if self.X.device.type == "cuda":     # run_concurrent: one workspace per stream
            key = (key, ops._stream_ptr(self.X))
        ent = self._ws.get(key)
        if ent is None or ent[0].shape[1] < rows or ent[0].shape[2] != cols:
            if ent is not None and ent[1]:      # a captured graph holds its address
                ops._GRAPH_HELD.append(ent[0])
            ent = [torch.zeros((3, rows, cols), dtype=torch.int16, device=self.X.device), False]
            self._ws[key] = ent
        if self.X.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            ent[1] = True
        return ent[0]

    def _stream_key(self):
        return ops._stream_ptr(self.X) if self.X.device.type == "cuda" else None

    def split_w(self, W: torch.Tensor, st: "_Batch"):
        """Planes of the spectra (times the count unit) for numer_gemm; call after every
        change of W that the W-solve epilogue did not emit (init, compaction)."""
        xp = self._planes()
        if xp is None:
            return None
        wpl = self._plane_buf("w", W.shape[0], xp.Gp)
        ops.split_planes(W, wpl[:, :W.shape[0]], col_mul=xp.unit)
        self.mark_w_fresh(W, st)
        return wpl

    def mark_w_fresh(self, W: torch.Tensor, st: "_Batch") -> None:
        """The current stream's "w" planes hold W of batch ``st`` at its current layout.
        Kept per stream (run_concurrent solves batches on several host threads, and a
        HIP-graph capture runs on a stream of its own whose buffer eager passes never
        wrote)."""
        self._w_fresh[self._stream_key()] = (W.data_ptr(), W.shape[0], st.uid,
                                             st.layout_version)

    def w_planes(self, W: torch.Tensor, st: "_Batch"):
        """The spectra planes, split only when the W-solve epilogue has not already
        written them for this W buffer / layout (solve(planes=...) below)."""
        xp = self._planes()
        if xp is None:
            return None
        if self._w_fresh.get(self._stream_key()) == (W.data_ptr(), W.shape[0], st.uid,
                                                     st.layout_version):
            return self._plane_buf("w", W.shape[0], xp.Gp)
        return self.split_w(W, st)

    def solve_planes(self, kind: str, rows: int, cols: int | None = None):
        """(planes buffer, column multiplier) a solve epilogue writes for the next GEMM:
        kind 'w' -> the spectra planes (genes on k, times the count unit); 'h' -> the
        usages planes of a chunk of ``cols`` cells (k padded to the GEMM's BK)."""
        xp = self._planes()
        if xp is None:
            return None, None
        if kind == "w":
            return self._plane_buf("w", rows, xp.Gp), xp.unit
        bk = ops.planes_bk(xp.pb)
        return self._plane_buf("h", rows, -(-cols // bk) * bk), None

    def numer_gemm(self, W: torch.Tensor, wpl, a: int, b: int) -> torch.Tensor:
        """numer = W X[a:b]^T (rows(W), b - a) -- split-precision MFMA when available."""
        xp = self._planes()
        if xp is None or wpl is None:
            self._need_x("the numerator GEMM without planes")
            return W @ self.X[a:b].t()
        out = torch.empty((W.shape[0], b - a), device=W.device, dtype=W.dtype)
        ops.gemm_planes(out, wpl[:ops.gemm_a_planes(xp.Gp)], xp.x[:, a:], W.shape[0], b - a,
                        xp.Gp)
        return out

    def stats_gemm(self, B: torch.Tensor, HT: torch.Tensor, a: int, b: int,
                   accumulate: bool, presplit: bool = False) -> None:
        """B (+)= HT[:, a:b] X[a:b]  (rows(HT), G) -- split-precision MFMA when available
        (and the chunk start is 8-aligned for the planes' k offset).  ``presplit``: the
        H-solve epilogue already wrote the usages planes (solve_planes('h'))."""
        xp = self._planes()
        if xp is None or a % 8:
            self._need_x("a statistics GEMM at a chunk start that is not 8-aligned")
            B.addmm_(HT[:, a:b], self.X[a:b], beta=1.0 if accumulate else 0.0)
            return
        bk = ops.planes_bk(xp.pb)
        kd = -(-(b - a) // bk) * bk
        hpl = self._plane_buf("h", HT.shape[0], kd)
        if not presplit:
            ops.split_planes(HT[:, a:b], hpl[:, :HT.shape[0]])
        ops.gemm_planes(B, hpl[:ops.gemm_a_planes(kd)], xp.xt[:, :, a:], HT.shape[0], xp.G, kd,
                        accumulate=accumulate, col_scale=xp.unit)

    def _need_x(self, what: str) -> None:
        if self._virtual:
            raise ValueError(f"PlanesOnlyX: {what} needs the fp32 matrix, which is not held "
                             "(online chunk starts must be multiples of 8)")

    def _mean(self) -> float:
        """Global mean of X (random init scale), one pass per solver."""
        if self._mean_x is None:
            self._mean_x = _global_mean(self.X, self.comm)
        return self._mean_x

    def run_concurrent(self, seeds, n_streams: int = 2, min_group: int = 8) -> NMFResult:
        """Split the replicates into ``n_streams`` groups solved concurrently, each on its
        own HIP stream (one host thread per stream).  One group's latency-bound inner solves
        then overlap another group's GEMMs; results are identical to ``run`` on each group.
        The cooperative solves of the groups share the co-residency budget
        (ops.coop_share), so their spin-waiting workgroups can always all be resident.

        Measured on the bench shape (100 replicates, 10k x 2k, K=10) this is SLOWER than
        one stream (2 streams 34 ms, 3: 40 ms, 4: 70 ms vs 19.9 ms): the halved coop
        budget lengthens the tail solves and the host threads contend for the GIL.  Kept
        opt-in (bench --streams) for shapes with few, long passes."""
        seeds = list(seeds)
        if (self.X.device.type != "cuda" or n_streams <= 1 or self.comm.is_distributed
                or len(seeds) < n_streams * min_group):
            return self.run(seeds)
        import concurrent.futures as cf

        bounds = np.linspace(0, len(seeds), n_streams + 1).astype(int)
        groups = [seeds[bounds[i]:bounds[i + 1]] for i in range(n_streams)]
        dev = self.X.device
        ops.coop_prepare(dev)   # device queries from the main thread (fail in workers)
        if self.beta == 2.0:
            self._planes()      # built once here, not raced by the worker threads
        main = torch.cuda.current_stream(dev)
        streams = [torch.cuda.Stream(dev) for _ in groups]
        for s_ in streams:
            s_.wait_stream(main)

        def work(i):
            from .nmf_graphs import _TLS

            torch.cuda.set_device(dev)
            _TLS.no_graphs = True            # eager passes in the worker threads
            with torch.cuda.stream(streams[i]), ops.coop_share(n_streams):
                return self.run(groups[i])

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(max_workers=n_streams) as ex:
            parts = list(ex.map(work, range(n_streams)))
        for s_ in streams:
            main.wait_stream(s_)
        stats = {"wall_s": time.perf_counter() - t0, "streams": n_streams,
                 "h_inner_iters": sum((p_.stats["h_inner_iters"] for p_ in parts), []),
                 "w_inner_iters": sum((p_.stats["w_inner_iters"] for p_ in parts), [])}
        return NMFResult(HT=torch.cat([p_.HT for p_ in parts]), W=torch.cat([p_.W for p_ in parts]),
                         err=np.concatenate([p_.err for p_ in parts]),
                         n_iter=np.concatenate([p_.n_iter for p_ in parts]),
                         converged=np.concatenate([p_.converged for p_ in parts]),
                         seeds=seeds, K=parts[0].K, stats=stats)

    # ------------------------------------------------------------------ helpers
    def _steps(self, N: int):
        if self.schedule is not None:
            return self.schedule
        c = max(1, int(self.opts.online_chunk_size))
        n_steps = self.comm.allreduce_max_int((N + c - 1) // c)
        return [[blk] for blk in _chunks(N, c, n_steps)]

    def _check_convergence(self, st: _Batch, err_now: torch.Tensor, step: int,
                           final: bool) -> None:
        """Host-side convergence step for the beta != 2 paths (errors computed on host)."""
        st.set_err(err_now, step, self.opts.tol, final)
        st.compact()

    def _init_err(self, st: _Batch) -> None:
        st.set_err(self.loss(st.HT, st.W, st.kpos if self.beta == 2.0 else st.K), 0,
                   self.opts.tol, False, init=True)

    def _init_err_frob(self, st: _Batch):
        """Initial Frobenius error of every replicate, on device (conv kernel, init mode).
        Returns the statistics (flat per-position K*K block A, rows B) of the initial H."""
        X = self.X
        G = X.shape[1]
        HT, W = st.views()
        rows, sq = st.rows_act, st.sq_act
        stats = torch.empty(rows * G + sq, device=X.device, dtype=X.dtype)
        B = stats[:rows * G].view(rows, G)
        A = stats[rows * G:]
        self.stats_gemm(B, HT, 0, X.shape[0], accumulate=False)
        for g in st.groups:
            ops.gram(g.rep3(HT), out=g.gram3(A))
        self.comm.allreduce_(stats)
        lin = torch.empty(st.n_act, device=X.device, dtype=torch.float32)
        quad = torch.empty_like(lin)
        for g in st.groups:
            W3 = g.rep3(W)
            lin[g.pos] = (g.rep3(B) * W3).sum(dim=(1, 2)).float()
            quad[g.pos] = (g.gram3(A) * ops.gram(W3)).sum(dim=(1, 2)).float()
        ops.conv_update(lin, quad, self.x_sq, st.state, st.n_act, 0, self.opts.tol, False,
                        init=True, gate=st.gate)
        return A, B

    # ------------------------------------------------------------------ loss (any beta)
    def loss(self, HT: torch.Tensor, W: torch.Tensor, K, row_chunk: int = 4096) -> torch.Tensor:
        """sqrt(2 * D_beta(X || H W)) per replicate (sklearn square_root=True), global.
        ``K`` is one rank for all replicates or one rank per replicate (rows in order)."""
        X = self.X
        N, G = X.shape
        if self.beta == 2.0:
            kk = np.full(W.shape[0] // int(K), int(K)) if np.isscalar(K) else np.asarray(K)
            # ||X||^2 - 2 <HT X, W> + <HT HT^T, W W^T>, per replicate
            B = HT @ X
            lin = torch.empty(kk.size, dtype=torch.float64, device=X.device)
            quad = torch.empty_like(lin)
            r0 = 0
            for i, k in enumerate(kk):
                rs = slice(r0, r0 + int(k))
                h, w = HT[rs], W[rs]
                lin[i] = (B[rs] * w).sum().double()
                quad[i] = ((h @ h.t()) * (w @ w.t())).sum().double()
                r0 = rs.stop
            lin = self.comm.allreduce_(lin.contiguous())
            quad = self.comm.allreduce_(quad.contiguous())
            return torch.sqrt(torch.clamp(self.x_sq - 2 * lin.cpu() + quad.cpu(), min=0.0))
        K = int(K)
        R = W.shape[0] // K
        W3 = W.view(R, K, G)
        tot = ops.beta_loss(X, HT.view(R, K, N), W3, self.beta, self.opts.eps)
        tot = tot.to(torch.float64).contiguous()
        self.comm.allreduce_(tot)
        return torch.sqrt(torch.clamp(2.0 * tot.cpu(), min=0.0))

    # ------------------------------------------------------------------ fused online step
    def _fused_ok(self, st: _Batch, steps) -> bool:
        """Whether the online Frobenius passes can run the FUSED step: GEMM -> pipelined
        H-solve -> GEMM -> pipelined W-solve with no reduction or Gram launch between them
        (split-K slabs summed by the consuming solve, the Grams passed between the solves
        as per-slice partials; solve_pipe.hip).  Needs the split-GEMM planes, MU without
        regularisation, the block-objective stop, one block per online step (8-aligned), a
        single process (the DP path all-reduces the statistics), K <= 64 and solves whose
        cooperative slices fit the pipelined kernel.  CNMF_FUSED_STEP=0 disables it."""
        o = self.opts
        if self.comm.is_distributed:
            # cell-sharded DP: every rank must take the same path (collective sequence)
            ok = self._fused_ok_local(st, steps, dp=True)
            return self.comm.allreduce_max_int(0 if ok else 1) == 0
        return self._fused_ok_local(st, steps, dp=False)

    def _fused_ok_local(self, st: _Batch, steps, dp: bool) -> bool:
        o = self.opts
        if (self.X.device.type != "cuda" or os.environ.get("CNMF_FUSED_STEP", "1") == "0"
                or ops._ENV["CNMF_SOLVE_PIPE"] == "0" or o.algo != "mu"
                or o.online_stats != "pass" or o.online_inner_conv != "loss"
                or any(v != 0.0 for v in (o.l1_H, o.l2_H, o.l1_W, o.l2_W))
                or self._planes() is None):
            return False
        if dp:
            # the reduce-scattered W-solve partitions the replicates of every K group of
            # the batch over the ranks (mixed-K batches: one packed exchange per group)
            if (os.environ.get("CNMF_DP_FUSED", "1") == "0"
                    or not hasattr(self.comm, "reduce_scatter_")):
                return False
        G = self.X.shape[1]
        for blocks in steps:
            if len(blocks) != 1 or blocks[0][0] % 8 or blocks[0][1] <= blocks[0][0]:
                return False
        dev = self.X.device
        for g in st.groups:
            for n in {b - a for (a, b), in steps} | {G}:
                if ops.pipe_slices(n, g.n, g.K, dev) is None:
                    return False
        return True

    def _fused_bufs(self, st: _Batch, steps) -> dict:
        """Per-layout workspaces of the fused step (allocated when the layout changes)."""
        xp = self._planes()
        dev = self.X.device
        rows, sq = st.rows_act, st.sq_act
        G = self.X.shape[1]
        cws = [b - a for (a, b), in steps]
        bk = ops.planes_bk(xp.pb)
        ks_n = max(ops.gemm_plan(rows, cw, xp.Gp, xp.pb)[1] for cw in cws)
        ks_b = max(ops.gemm_plan(rows, G, -(-cw // bk) * bk, xp.pb)[1] for cw in cws)
        S = ops.kCoopMaxSlices
        ngp = sum(g.n * S * g.K * g.K for g in st.groups)
        kd_max = max(-(-cw // bk) * bk for cw in cws)
        fb = {
            "wpl": torch.zeros((3, rows, xp.Gp), device=dev, dtype=torch.int16),
            "hpl": torch.zeros((3, rows, kd_max), device=dev, dtype=torch.int16),
            "wpl_key": None,
            "slabN": torch.empty(ks_n * rows * max(cws), device=dev, dtype=torch.float32),
            "slabB": torch.empty(ks_b * rows * G, device=dev, dtype=torch.float32),
            "B": torch.empty((rows, G), device=dev, dtype=torch.float32),
            "A": [torch.empty(sq, device=dev, dtype=torch.float32) for _ in range(2)],
            "WWp": torch.empty(max(ngp, 1), device=dev, dtype=torch.float32),
            "HHp": torch.empty(max(ngp, 1), device=dev, dtype=torch.float32),
            "lin": torch.zeros(st.n_act, device=dev, dtype=torch.float32),
            "quad": torch.zeros(st.n_act, device=dev, dtype=torch.float32),
            "wwp_n": {}, "hhp_n": {}, "wwp_key": None,
        }
        off = 0
        fb["parts"] = {}
        for g in st.groups:
            m = g.n * S * g.K * g.K
            fb["parts"][g.p0] = (lambda t, o_=off, g_=g: t[o_:o_ + g_.n * S * g_.K * g_.K]
                                 .view(g_.n, S, g_.K, g_.K))
            off += m
        if os.environ.get("CNMF_HOST_FLAGS", "1") != "0":
            # the passes' active flags, stored by conv_update through the host mapping into
            # two alternating slots, and its launch counter (device, plus the host's mirror)
            fb["hflags"] = torch.ones((2, st.n_act), dtype=torch.int32, pin_memory=True)
            fb["hcnt"] = torch.zeros(1, dtype=torch.int32, device=dev)
            fb["hcnt_host"] = [0]
        return fb

    def _fused_prep(self, st: _Batch, fb: dict, keep_slices: bool):
        """The fused pass's operands that depend on W when W changed outside the fused
        W-solve (init, compaction, an unfused pass): the W W^T partials (the Gram kernel's
        full Gram in partial slot 0) and the spectra's bf16 planes.  ``keep_slices``: the
        pass will be a graph replay captured with the W-solve's slice count S_w as the
        number of partials to sum -- slots 1..S_w-1 are zeroed instead of the count
        dropping to 1 (the sum is the same Gram, bitwise).  Returns the W key."""
        xp = self._planes()
        HT, W = st.views()
        active = st.active_mask()
        wkey = (W.data_ptr(), st.rows_act, st.uid, st.layout_version)
        if fb["wwp_key"] != wkey:
            for g in st.groups:
                parts = fb["parts"][g.p0](fb["WWp"])
                parts[:, 0].copy_(ops.gram(g.rep3(W), active=active[g.pos]))
                n_s = fb["wwp_n"].get(g.p0, 1) if keep_slices else 1
                if n_s > 1:
                    parts[:, 1:n_s].zero_()
                fb["wwp_n"][g.p0] = n_s
            if keep_slices:
                fb["wwp_key"] = wkey
        if fb["wpl_key"] != wkey:      # spectra planes: split here only after such a change
            ops.split_planes(W, fb["wpl"], col_mul=xp.unit)
            fb["wpl_key"] = wkey
        return wkey

    def _enqueue_fused(self, st: _Batch, steps, cur: dict) -> None:
        """Enqueue one single-process fused pass (_enqueue_fused_pass) and point
        ``st.host_flags`` at the host-mapped slot its conv_update stores the active flags
        in (the layout's launch count, mirrored on the host, picks the slot)."""
        self._enqueue_fused_pass(st, steps, cur)
        fb = cur["fb"]
        if "hflags" in fb:
            c = fb["hcnt_host"][0]
            fb["hcnt_host"][0] = c + 1
            st.host_flags = fb["hflags"][c & 1]

    def _enqueue_fused_pass(self, st: _Batch, steps, cur: dict) -> None:
        """Enqueue one single-process fused pass: from the layout's captured graph when
        the batch has an arena (captured on the layout's second pass; a layout an earlier
        run captured replays from its first, with only the W-dependent operands rebuilt
        eagerly), else eagerly.  ``cur`` carries the layout's workspaces between calls."""
        key = (st.uid, st.layout_version)
        if cur["key"] != key or cur.pop("fresh", False):
            if cur["key"] != key:
                sl = cur["sl"] = self._slot(st, steps) if st.graphs else None
                cur["fb"] = sl["fb"] if sl is not None else self._fused_bufs(st, steps)
                cur["key"] = key
                if "hflags" in cur["fb"]:
                    # the layout's first pass in this run: the flag kernel's launch counter
                    # and the host's mirror restart together (whatever an earlier run, or
                    # one that raised, left behind), ahead of this pass's launch
                    cur["fb"]["hcnt"].zero_()
                    cur["fb"]["hcnt_host"][0] = 0
            sl = cur["sl"]
            if sl is not None and sl["graph"] is not None and _LAYOUT_REPLAY:
                self._fused_prep(st, cur["fb"], keep_slices=True)
                sl["graph"].replay()
            else:
                self._fused_pass(st, steps, cur["fb"])
            return
        sl = cur["sl"]
        if sl is None or not self._replay_slot(sl, st, steps):
            self._fused_pass(st, steps, cur["fb"])

    def _fused_pass(self, st: _Batch, steps, fb: dict, final: bool = False) -> None:
        """One online pass of the fused step (see _fused_ok); same updates, stopping rules
        and statistics as the unfused pass -- the split-K sums and the accumulation of
        B / A are bitwise the unfused ones, the Grams are summed per slice instead of per
        Gram-kernel workgroup (fp32 rounding order only).  The pass limit is applied per
        replicate on the device (conv_update max_pass), so every pass -- the last one
        included -- is the same launch sequence and replays from one graph."""
        o = self.opts
        xp = self._planes()
        G = self.X.shape[1]
        HT, W = st.views()
        rows = st.rows_act
        groups = st.groups
        active = st.active_mask()
        n = st.n_act
        h_it, w_it = st.h_iters[:n], st.w_iters[:n]
        bk = ops.planes_bk(xp.pb)
        slabN, slabB, B = fb["slabN"], fb["slabB"], fb["B"]
        wkey = self._fused_prep(st, fb, keep_slices=False)
        last_s = len(steps) - 1
        wpl = fb["wpl"]
        wpl_n = ops.gemm_a_planes(xp.Gp)
        for s_, ((a, b),) in enumerate(steps):
            cw = b - a
            ks_n = ops.gemm_planes(None, wpl[:wpl_n], xp.x[:, a:], rows, cw, xp.Gp,
                                   raw_slab=slabN, raw_max=_FUSED_MAX_SLABS, gate=st.gate)
            kd = -(-cw // bk) * bk
            hpl = fb["hpl"][:, :, :kd]
            hpl_n = ops.gemm_a_planes(kd)
            hcols = HT[:, a:b]
            for g in groups:
                numer = slabN.as_strided((g.n, g.K, cw), (g.K * cw, cw, 1), g.r0 * cw)
                fb["hhp_n"][g.p0] = ops.solve(
                    "mu", g.rep3(hcols), numer, None, max_iter=o.online_chunk_max_iter,
                    tol=o.online_h_tol, eps=o.eps, iters_out=h_it[g.pos], conv_mode=1,
                    check_every=o.inner_check_every, active=active[g.pos],
                    planes=hpl[:, g.rows], planes_n=hpl_n, numer_slabs=ks_n,
                    numer_slab_stride=rows * cw,
                    gram_parts=fb["parts"][g.p0](fb["WWp"]), gram_parts_n=fb["wwp_n"][g.p0],
                    gram_parts_out=fb["parts"][g.p0](fb["HHp"]), coop_device_gen=True)
            ks_b = ops.gemm_planes(None, hpl[:hpl_n], xp.xt[:, :, a:], rows, G, kd,
                                   raw_slab=slabB, raw_max=_FUSED_MAX_SLABS)
            last = s_ == last_s
            A_in, A_out = fb["A"][(s_ + 1) % 2], fb["A"][s_ % 2]
            for g in groups:
                numer = slabB.as_strided((g.n, g.K, G), (g.K * G, G, 1), g.r0 * G)
                fb["wwp_n"][g.p0] = ops.solve(
                    "mu", g.rep3(W), numer, None if s_ == 0 else g.gram3(A_in),
                    max_iter=o.online_chunk_max_iter, tol=o.online_w_tol, eps=o.eps,
                    lin_out=fb["lin"][g.pos] if last else None,
                    quad_out=fb["quad"][g.pos] if last else None,
                    iters_out=w_it[g.pos], conv_mode=1, check_every=o.inner_check_every,
                    active=active[g.pos], planes=wpl[:, g.rows], planes_colmul=xp.unit,
                    planes_n=wpl_n, numer_slabs=ks_b, numer_slab_stride=rows * G,
                    numer_scale=xp.unit, numer_base=None if s_ == 0 else g.rep3(B),
                    numer_out=None if last else g.rep3(B),
                    gram_parts=fb["parts"][g.p0](fb["HHp"]), gram_parts_n=fb["hhp_n"][g.p0],
                    gram_out=None if last else g.gram3(A_out),
                    gram_parts_out=fb["parts"][g.p0](fb["WWp"]), coop_device_gen=True)
            fb["wwp_key"] = fb["wpl_key"] = wkey
        ops.conv_update(fb["lin"], fb["quad"], self.x_sq, {k: v[:n] for k, v in st.state.items()},
                        n, -1, o.tol, final=final, gate=st.gate,
                        max_pass=int(o.online_max_pass),
                        host_flags=(fb["hflags"], fb["hcnt"]) if "hflags" in fb else None)
        if st.feed is not None:        # streaming: harvest / refill in this pass (stream.hip)
            self._stream_swap_dev(st, fb)

    # ------------------------------------------------------------------ online frobenius
    def _online_frob(self, st: _Batch) -> None:
        o, comm = self.opts, self.comm
        X = self.X
        N, G = X.shape
        dev, dt = X.device, X.dtype
        steps = self._steps(N)
        algo = o.algo
        cmode = 1 if o.online_inner_conv == "loss" else 0
        exact = o.online_stats == "exact"
        dist = comm.is_distributed
        A0, B0 = self._init_err_frob(st)
        if exact:
            st.A, st.B = A0.clone(), B0.clone()
        del A0, B0
        max_pass = int(o.online_max_pass)
        n_alloc = None
        graphs = _graphs_enabled(X) and not dist
        graph, graph_key, last_key = None, None, None
        fused = self._fused_ok(st, steps)
        # DP fused: the batch keeps one layout (no host compaction: 2.0 never fires) -- the
        # DP W-solve owns a fixed partition and only its rows of W are fresh
        dp_fused = fused and dist
        pipe = _PassPipeline(st, compact_frac=2.0 if dp_fused else None)
        fcur = {"fb": None, "key": None, "sl": None}
        if fused and st.feed is not None:
            self._stream_loop(st, steps, fcur)
            return
        for p in range(max_pass):
            n = st.n_act
            if n == 0:
                break
            if fused:
                if dp_fused:
                    key = (st.uid, st.layout_version)
                    if fcur["key"] != key:
                        fcur["fb"], fcur["key"] = self._fused_bufs_dp(st, steps), key
                    self._fused_pass_dp(st, steps, fcur["fb"], final=p + 1 == max_pass)
                else:
                    self._enqueue_fused(st, steps, fcur)
                if not pipe.after_enqueue():
                    break
                continue
            rows, sq = st.rows_act, st.sq_act
            if (rows, sq, n) != n_alloc:   # (re)allocate per-layout workspaces, not per pass
                n_alloc = (rows, sq, n)
                flat = torch.empty(rows * G + sq, device=dev, dtype=dt)
                dB = flat[:rows * G].view(rows, G)
                dA = flat[rows * G:]
                if not exact:
                    A = torch.empty(sq, device=dev, dtype=dt)
                    B = torch.empty((rows, G), device=dev, dtype=dt)
                lin = torch.zeros(n, device=dev, dtype=torch.float32)
                quad = torch.zeros(n, device=dev, dtype=torch.float32)
                wwt_buf = torch.empty(sq, device=dev, dtype=dt)
            final = p + 1 == max_pass

            def enqueue_pass(pass_arg: int, final: bool) -> None:
                HT, W = st.views()
                if exact:
                    A_, B_ = st.A[:sq], st.B[:rows]
                else:
                    A_, B_ = A, B
                    if dist:        # single process: the pass's first chunk overwrites
                        A_.zero_()
                        B_.zero_()
                pass_first = True
                active = st.active_mask()
                h_it = st.h_iters[:n]
                w_it = st.w_iters[:n]
                groups = st.groups
                for s_, blocks in enumerate(steps):
                    # DP: increments go to the flat buffer (one all-reduce per step); single
                    # process: GEMMs accumulate straight into A / B (beta = 1)
                    accA, accB = (dA, dB) if dist else (A_, B_)
                    first = True
                    wpl = None if exact else self.w_planes(W, st)  # the last W-solve's
                    for (a, b) in blocks:
                        cw = b - a
                        if cw <= 0:
                            continue
                        xc = X[a:b]
                        hcols = HT[:, a:b]                               # (rows, cw) strided
                        h_old = hcols.clone() if exact else None
                        numerT = self.numer_gemm(W, wpl, a, b)   # ONE GEMM, every K
                        # the H-solve epilogue writes the usages' bf16 planes for the
                        # statistics GEMM (no separate split pass), unless unaligned
                        hpl, _ = (None, None) if (exact or a % 8) else \
                            self.solve_planes("h", rows, b - a)
                        hpl_n = 3 if hpl is None else ops.gemm_a_planes(hpl.shape[2])
                        for g in groups:
                            ga = active[g.pos]
                            # W W^T: its own Gram launch (forming it in the matrix-core
                            # solve's prologue, ops.solve gram_of, measured slower: every
                            # usage-slice workgroup re-reads W at L2 latency;
                            # profiles/README.md)
                            WWT = ops.gram(g.rep3(W), out=g.gram3(wwt_buf), active=ga)
                            _inner_solve(algo, g.rep3(hcols), g.rep3(numerT), WWT,
                                         max_iter=o.online_chunk_max_iter, tol=o.online_h_tol,
                                         l1_den=o.l1_H, l2=o.l2_H, eps=o.eps,
                                         iters_out=h_it[g.pos], conv_mode=cmode,
                                         check_every=o.inner_check_every, active=ga,
                                         planes=None if hpl is None else hpl[:, g.rows],
                                         planes_n=hpl_n)
                        if exact:
                            # replace the chunk's old contribution: d = h_new - h_old
                            for g in groups:
                                hv, ho = g.rep3(hcols), g.rep3(h_old)
                                hh = torch.bmm(hv, hv.transpose(1, 2))
                                hh -= torch.bmm(ho, ho.transpose(1, 2))
                                if dist and first:
                                    g.gram3(accA).copy_(hh)
                                else:
                                    g.gram3(accA).add_(hh)
                            hlhs = h_old.neg_().add_(hcols)
                            accB.addmm_(hlhs, xc, beta=0.0 if (dist and first) else 1.0)
                        else:
                            if (dist and first) or (not dist and pass_first):
                                self.stats_gemm(accB, HT, a, b, False,   # B = h^T x, every K
                                                presplit=hpl is not None)
                                for g in groups:                       # A = h^T h
                                    ops.gram(g.rep3(hcols), out=g.gram3(accA),
                                             active=None if dist else active[g.pos])
                            else:
                                self.stats_gemm(accB, HT, a, b, True,   # B += h^T x
                                                presplit=hpl is not None)
                                for g in groups:                       # A += h^T h
                                    ops.gram(g.rep3(hcols), out=g.gram3(accA),
                                             accumulate=True, active=active[g.pos])
                        first = False
                        pass_first = False
                    if dist:
                        if first:
                            flat.zero_()
                        comm.allreduce_(flat)
                        B_ += dB
                        A_ += dA
                    last = s_ == len(steps) - 1
                    wpl_out, unit = (None, None) if exact else self.solve_planes("w", rows)
                    wpl_n = 3 if wpl_out is None else ops.gemm_a_planes(wpl_out.shape[2])
                    for g in groups:
                        _inner_solve(algo, g.rep3(W), g.rep3(B_), g.gram3(A_),
                                     max_iter=o.online_chunk_max_iter, tol=o.online_w_tol,
                                     l1_den=o.l1_W, l2=o.l2_W, eps=o.eps,
                                     lin_out=lin[g.pos] if last else None,
                                     quad_out=quad[g.pos] if last else None,
                                     iters_out=w_it[g.pos], conv_mode=cmode,
                                     check_every=o.inner_check_every, active=active[g.pos],
                                     planes=None if wpl_out is None else wpl_out[:, g.rows],
                                     planes_colmul=unit, planes_n=wpl_n)
                    if wpl_out is not None:
                        self.mark_w_fresh(W, st)
                ops.conv_update(lin, quad, self.x_sq, {k: v[:n] for k, v in st.state.items()},
                                n, pass_arg, o.tol, final=final)

            # A pass is a fixed sequence (~4 launches per chunk) for a given batch layout:
            # after one eager pass with the layout (warms the GEMM heuristics and the
            # workspaces) it is captured once into a HIP graph and replayed while the
            # layout holds -- the host then spends one launch per pass, not ~50.
            key = (n, st.layout_version)
            if graphs and not final and key == last_key:
                if graph_key != key:
                    try:
                        graph = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                            enqueue_pass(-1, False)
                        graph_key = key
                    except RuntimeError:          # capture unsupported here: stay eager
                        graphs, graph = False, None
                if graph is not None:
                    graph.replay()
                    # the replay's W-solves wrote the capture stream's planes: this
                    # stream's copy now holds an older W
                    self._w_fresh.pop(self._stream_key(), None)
                else:
                    enqueue_pass(-1, final)
            else:
                t_h = time.perf_counter()
                enqueue_pass(-1, final)
                if self.profile:
                    self.timings.setdefault("host_pass", []).append(
                        (n, time.perf_counter() - t_h))
            last_key = key
            t_w = time.perf_counter()
            if not pipe.after_enqueue():
                break
            if self.profile:
                self.timings.setdefault("wait_pass", []).append((n, time.perf_counter() - t_w))
        if graph is not None:
            torch.cuda.current_stream().synchronize()
        if fused and dist and fcur["fb"] is not None:
            self._dp_gather_w(st, fcur["fb"])

    # ------------------------------------------------------------------ batch frobenius
    def _batch_frob(self, st: _Batch) -> None:
        o, comm = self.opts, self.comm
        X = self.X
        N, G = X.shape
        dev, dt = X.device, X.dtype
        self._init_err_frob(st)
        inner = o.algo == "halsvar"          # HALS loops to tolerance; else one sweep
        h_iter = o.batch_hals_max_iter if inner else 1
        h_tol = o.batch_hals_tol if inner else -1.0
        max_it = int(o.batch_max_iter)
        every = max(1, int(o.loss_every))
        pipe = _PassPipeline(st)
        n_alloc = None
        for it in range(max_it):
            n = st.n_act
            if n == 0:
                break
            rows, sq = st.rows_act, st.sq_act
            if (rows, sq, n) != n_alloc:
                n_alloc = (rows, sq, n)
                flat = torch.empty(rows * G + sq, device=dev, dtype=dt)
                B = flat[:rows * G].view(rows, G)
                A = flat[rows * G:]
                lin = torch.zeros(n, device=dev, dtype=torch.float32)
                quad = torch.zeros(n, device=dev, dtype=torch.float32)
                wwt = torch.empty(sq, device=dev, dtype=dt)
            HT, W = st.views()
            active = st.active_mask()
            # H-step over all local cells: one numerator GEMM for every K
            numerT = self.numer_gemm(W, self.w_planes(W, st), 0, N)
            nsplit = 1 if inner else max(1, (N + 8191) // 8192)
            hpl, _ = self.solve_planes("h", rows, N)
            for g in st.groups:
                WWT = ops.gram(g.rep3(W), out=g.gram3(wwt), active=active[g.pos])
                _inner_solve(o.algo, g.rep3(HT), g.rep3(numerT), WWT,
                             max_iter=h_iter, tol=h_tol, l1_den=o.l1_H, l2=o.l2_H, eps=o.eps,
                             nsplit=nsplit, active=active[g.pos],
                             iters_out=st.h_iters[g.pos],
                             planes=None if hpl is None else hpl[:, g.rows])
            del numerT
            # W-step from the new H
            self.stats_gemm(B, HT, 0, N, accumulate=False, presplit=hpl is not None)
            for g in st.groups:
                ops.gram(g.rep3(HT), out=g.gram3(A))
            comm.allreduce_(flat)
            check = (it + 1) % every == 0 or it + 1 == max_it
            wpl_out, unit = self.solve_planes("w", rows)
            for g in st.groups:
                _inner_solve(o.algo, g.rep3(W), g.rep3(B), g.gram3(A),
                             max_iter=h_iter, tol=h_tol, l1_den=o.l1_W, l2=o.l2_W, eps=o.eps,
                             lin_out=lin[g.pos] if check else None,
                             quad_out=quad[g.pos] if check else None,
                             active=active[g.pos], iters_out=st.w_iters[g.pos],
                             planes=None if wpl_out is None else wpl_out[:, g.rows],
                             planes_colmul=unit)
            if wpl_out is not None:
                self.mark_w_fresh(W, st)
            if check:
                ops.conv_update(lin, quad, self.x_sq, {k: v[:n] for k, v in st.state.items()},
                                n, it + 1, o.tol, final=(it + 1 == max_it))
                if not pipe.after_enqueue():
                    break



def _as(t: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    """Contiguous copy/view of ``t`` in ``dt`` (solve kernels take dense grams)."""
    return t.contiguous() if t.dtype == dt else t.to(dt).contiguous()



# =============================================================================== api
def run_nmf_batch(X, n_components: int, seeds, comm=None, row_offset: int = 0, device=None,
                  **kwargs) -> NMFResult:
    """Factorise ``X`` (cells x genes) once per seed; see module docstring."""
    if not isinstance(X, torch.Tensor):
        X = torch.as_tensor(np.asarray(X))
    if device is not None:
        X = X.to(device)
    opts = NMFOptions.from_kwargs(n_components, **kwargs)
    return NMFBatchSolver(X, opts, comm=comm, row_offset=row_offset).run(list(seeds))



def run_nmf(X, n_components: int, init: str = "random", beta_loss="frobenius", algo: str = "mu",
            mode: str = "online", tol: float = 1e-4, n_jobs: int = -1, random_state: int = 0,
            use_gpu: bool = False, alpha_W: float = 0.0, l1_ratio_W: float = 0.0,
            alpha_H: float = 0.0, l1_ratio_H: float = 0.0, fp_precision: str = "float",
            batch_max_iter: int = 500, batch_hals_tol: float = 0.05,
            batch_hals_max_iter: int = 200, online_max_pass: int = 20,
            online_chunk_size: int = 5000, online_chunk_max_iter: int = 200,
            online_h_tol: float = 0.05, online_w_tol: float = 0.05):
    """Single-replicate drop-in for nmf-torch's ``run_nmf`` (cnmf.py:17, 819).

    Returns (H: N x K usages, W: K x G spectra, err) as numpy arrays.  ``n_jobs`` only
    sets CPU threads; ``use_gpu`` selects the current HIP device.
    """
    if n_jobs is not None and n_jobs > 0:
        torch.set_num_threads(int(n_jobs))
    dev = torch.device("cuda") if (use_gpu and torch.cuda.is_available()) else torch.device("cpu")
    res = run_nmf_batch(X, n_components, [int(random_state)], device=dev, init=init,
                        beta_loss=beta_loss, algo=algo, mode=mode, tol=tol, alpha_W=alpha_W,
                        l1_ratio_W=l1_ratio_W, alpha_H=alpha_H, l1_ratio_H=l1_ratio_H,
                        fp_precision=fp_precision, batch_max_iter=batch_max_iter,
                        batch_hals_tol=batch_hals_tol, batch_hals_max_iter=batch_hals_max_iter,
                        online_max_pass=online_max_pass, online_chunk_size=online_chunk_size,
                        online_chunk_max_iter=online_chunk_max_iter, online_h_tol=online_h_tol,
                        online_w_tol=online_w_tol)
    H = res.usages(0).cpu().numpy()
    W = res.spectra(0).cpu().numpy()
    return H, W, float(res.err[0])

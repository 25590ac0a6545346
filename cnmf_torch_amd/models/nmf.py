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
"""
from __future__ import annotations

import collections
import itertools
import math
import os
import time
import weakref
from dataclasses import dataclass, field, asdict

import numpy as np
import torch

from .. import ops
from .bpp import nnls_bpp, objective_terms as bpp_objective_terms
from ..parallel.comm import LocalComm
from ..utils import rng
from ..utils.log import get_logger

log = get_logger("cnmf_torch_amd.nmf")

BETA_LOSS = {"frobenius": 2.0, "kullback-leibler": 1.0, "itakura-saito": 0.0}


def beta_value(beta_loss) -> float:
    if isinstance(beta_loss, str):
        if beta_loss not in BETA_LOSS:
            raise ValueError(f"beta_loss must be one of {list(BETA_LOSS)} or a number, got {beta_loss!r}")
        return BETA_LOSS[beta_loss]
    return float(beta_loss)


@dataclass
class NMFOptions:
    n_components: int
    init: str = "random"
    beta_loss: object = "frobenius"
    algo: str = "mu"
    mode: str = "online"
    tol: float = 1e-4
    alpha_W: float = 0.0        # spectra regularisation (nmf-torch W = cnmf spectra)
    l1_ratio_W: float = 0.0
    alpha_H: float = 0.0        # usage regularisation
    l1_ratio_H: float = 0.0
    fp_precision: str = "float"
    batch_max_iter: int = 500
    batch_hals_tol: float = 0.05
    batch_hals_max_iter: int = 200
    online_max_pass: int = 20
    online_chunk_size: int = 5000
    online_chunk_max_iter: int = 200
    online_h_tol: float = 0.05
    online_w_tol: float = 0.05
    online_stats: str = "pass"  # "pass": A,B reset each pass (Mairal); "exact": A=H^T H, B=H^T X of current H
    online_inner_conv: str = "loss"  # 'loss': block objective every inner_check_every steps; 'iterate'
    inner_check_every: int = 10
    # beta != 2 online spectra iterations stop on the relative iterate change (the block
    # objective would cost a pass over the chunk per evaluation); online_w_tol's 0.05 stops
    # them after one step, which left online KL/IS unconverged after 20 passes
    online_beta_w_tol: float = 5e-3
    loss_every: int = 10
    eps: float = 1e-16
    # KL on the GPU runs its MU statistics over the non-zeros only (CSR kernels,
    # sparse_kl.hip) when X has at most this fraction of non-zero entries; 0 disables.
    # CNMF_KL_SPARSE=1 / 0 forces / disables it.  Measured crossover (profiles/r4h_kl_*,
    # r4c_kl_*; CSR vs dense rep/s): 8 % 564 / 381, 15 % 403 / 365, 25 % 290 / 348,
    # 35 % 228 / 338 -- equal near 19 %; at the headline's 47 % the dense kernels win
    kl_sparse_density: float = 0.18

    @classmethod
    def from_kwargs(cls, n_components: int, **kw) -> "NMFOptions":
        names = set(cls.__dataclass_fields__)
        return cls(n_components=int(n_components), **{k: v for k, v in kw.items() if k in names})

    def validate(self) -> None:
        if self.algo not in ("mu", "hals", "halsvar", "bpp"):
            raise ValueError(f"algo must be 'mu', 'hals', 'halsvar' or 'bpp', got {self.algo!r}")
        if self.mode not in ("online", "batch"):
            raise ValueError(f"mode must be 'online' or 'batch', got {self.mode!r}")
        if self.algo in ("hals", "halsvar", "bpp") and beta_value(self.beta_loss) != 2.0:
            raise ValueError(f"{self.algo.upper()} is defined for the Frobenius loss only")
        if self.init not in ("random", "nndsvd", "nndsvda", "nndsvdar"):
            raise ValueError(f"unsupported init {self.init!r}")
        if self.fp_precision not in ("float", "double"):
            raise ValueError("fp_precision must be 'float' or 'double'")

    @property
    def dtype(self) -> torch.dtype:
        return torch.float32 if self.fp_precision == "float" else torch.float64

    @property
    def l1_W(self):
        return self.alpha_W * self.l1_ratio_W

    @property
    def l2_W(self):
        return self.alpha_W * (1.0 - self.l1_ratio_W)

    @property
    def l1_H(self):
        return self.alpha_H * self.l1_ratio_H

    @property
    def l2_H(self):
        return self.alpha_H * (1.0 - self.l1_ratio_H)


@dataclass
class NMFResult:
    """Batch result in the callers' replicate order.  ``HT`` (sum_r K_r, N_local) holds the
    usages transposed and ``W`` (sum_r K_r, G) the spectra; replicate r owns rows
    ``offs[r] : offs[r] + ks[r]`` of both.  ``K`` is the common K of a single-K batch
    (None for a mixed-K batch)."""

    HT: torch.Tensor
    W: torch.Tensor
    err: np.ndarray
    n_iter: np.ndarray
    converged: np.ndarray
    seeds: list
    K: int | None
    stats: dict = field(default_factory=dict)
    ks: np.ndarray | None = None

    def __post_init__(self):
        if self.ks is None:
            self.ks = np.full(len(self.seeds), int(self.K), dtype=np.int64)
        self.ks = np.asarray(self.ks, dtype=np.int64)
        self.offs = np.concatenate([[0], np.cumsum(self.ks)[:-1]]).astype(np.int64)

    def rows(self, r: int) -> slice:
        return slice(int(self.offs[r]), int(self.offs[r] + self.ks[r]))

    def usages(self, r: int) -> torch.Tensor:
        return self.HT[self.rows(r)].t()

    def spectra(self, r: int) -> torch.Tensor:
        return self.W[self.rows(r)]


# =============================================================================== init
def _global_mean(X: torch.Tensor, comm) -> float:
    # float64 accumulation over row blocks (a dtype= reduction would copy X to float64)
    s = comm.allreduce_scalar(sum(float(X[a:a + (1 << 16)].sum(dtype=torch.float64))
                                  for a in range(0, X.shape[0], 1 << 16)))
    n = comm.allreduce_scalar(float(X.numel()))
    return s / max(n, 1.0)


def _nndsvd(X: torch.Tensor, K: int, variant: str, comm, eps: float = 1e-6, seed: int = 0):
    """sklearn's NNDSVD init (sklearn/decomposition/_nmf.py:316-366) via the Gram
    eigendecomposition, so it works on a cell-sharded X (only G x G and norms are
    all-reduced).  Returns (H (N_loc x K), W (K x G)) in X's dtype."""
    rows = 1 << 16    # float64 row blocks: never a full float64 copy of X
    G = X.shape[1]
    C = torch.zeros((G, G), dtype=torch.float64, device=X.device)
    for a in range(0, X.shape[0], rows):
        xb = X[a:a + rows].to(torch.float64)
        C.addmm_(xb.t(), xb)
    comm.allreduce_(C)
    evals, evecs = torch.linalg.eigh(C)
    order = torch.argsort(evals, descending=True)[:K]
    S = torch.sqrt(torch.clamp(evals[order], min=0.0))
    V = evecs[:, order].t()                       # K x G
    U = torch.cat([X[a:a + rows].to(torch.float64) @ V.t()
                   for a in range(0, X.shape[0], rows)]) if X.shape[0] else \
        torch.zeros((0, K), dtype=torch.float64, device=X.device)
    U = U / torch.clamp(S, min=1e-300)            # N_loc x K
    Wsk = torch.zeros_like(U)                     # sklearn W = usages
    Hsk = torch.zeros_like(V)                     # sklearn H = spectra
    Wsk[:, 0] = torch.sqrt(S[0]) * torch.abs(U[:, 0])
    Hsk[0, :] = torch.sqrt(S[0]) * torch.abs(V[0, :])
    for j in range(1, K):
        x, y = U[:, j], V[j, :]
        xp, yp = torch.clamp(x, min=0), torch.clamp(y, min=0)
        xn, yn = torch.clamp(-x, min=0), torch.clamp(-y, min=0)
        xpn = math.sqrt(comm.allreduce_scalar(float((xp * xp).sum())))
        xnn = math.sqrt(comm.allreduce_scalar(float((xn * xn).sum())))
        ypn, ynn = float(torch.linalg.norm(yp)), float(torch.linalg.norm(yn))
        mp, mn = xpn * ypn, xnn * ynn
        if mp > mn:
            u, v, sigma = xp / max(xpn, 1e-300), yp / max(ypn, 1e-300), mp
        else:
            u, v, sigma = xn / max(xnn, 1e-300), yn / max(ynn, 1e-300), mn
        lbd = math.sqrt(float(S[j]) * sigma)
        Wsk[:, j] = lbd * u
        Hsk[j, :] = lbd * v
    Wsk[Wsk < eps] = 0
    Hsk[Hsk < eps] = 0
    if variant in ("nndsvda", "nndsvdar"):
        avg = _global_mean(X, comm)
        if variant == "nndsvda":
            Wsk[Wsk == 0] = avg
            Hsk[Hsk == 0] = avg
        else:
            g = torch.Generator(device="cpu").manual_seed(int(seed))
            a = avg / 100.0
            rw = torch.abs(torch.randn(Wsk.shape, generator=g, dtype=torch.float64)) * a
            rh = torch.abs(torch.randn(Hsk.shape, generator=g, dtype=torch.float64)) * a
            Wsk = torch.where(Wsk == 0, rw.to(Wsk.device), Wsk)
            Hsk = torch.where(Hsk == 0, rh.to(Hsk.device), Hsk)
    return Wsk.to(X.dtype), Hsk.to(X.dtype)


def init_into(HT: torch.Tensor, W: torch.Tensor, X: torch.Tensor, K: int, seeds,
              init: str = "random", comm=None, row_offset: int = 0,
              mean: float | None = None, row_map=None) -> None:
    """Fill the row blocks HT (R*K x N_loc) and W (R*K x G) with the initial factors of R
    replicates of rank K (contiguous row blocks of a possibly larger ragged batch).

    random: |N(0,1)| * sqrt(mean(X)/K) from Philox keyed by each replicate's seed
    (H stream 0 over the canonical N x K matrix, W stream 1 over K x G), identical on
    every device and for every rank/batch placement.  ``mean`` (global mean of X) may be
    passed to skip its pass over X.  ``row_map`` [(local_start, local_stop,
    global_start)] places non-contiguous global rows (a chunk-interleaved DP shard);
    default: local rows are global rows ``row_offset + i``."""
    comm = comm or LocalComm()
    R = len(seeds)
    N, G = X.shape
    if init == "random":
        if mean is None:
            mean = _global_mean(X, comm)
        avg = math.sqrt(mean / K)
        seeds_t = torch.tensor([int(s) for s in seeds], dtype=torch.int64)
        if HT.device.type == "cuda":
            # one async copy from pinned memory and a device fill, shared by the H and W
            # draws (four pageable copies, each blocking the host, led every run)
            seeds_t = seeds_t.pin_memory().to(HT.device, non_blocking=True)
            scales = torch.full((R,), avg, dtype=torch.float32, device=HT.device)
        else:
            scales = torch.full((R,), avg, dtype=torch.float32)
        ld = HT.stride(0)
        for la, lb, ga in (row_map if row_map is not None else [(0, N, row_offset)]):
            if lb > la:
                # HT columns [la, lb) viewed as (R, n, K): element (r, j, k) -> HT[r*K+k, la+j]
                ops.philox_fill(HT.as_strided((R, lb - la, K), (K * ld, 1, ld),
                                              HT.storage_offset() + la),
                                seeds_t, scales, rng.STREAM_H, 0, ga)
        ops.philox_fill(W.view(R, K, G), seeds_t, scales, rng.STREAM_W, 0, 0)
    else:
        Hn, Wn = _nndsvd(X, K, init, comm, seed=int(seeds[0]) if len(seeds) else 0)
        for r in range(R):
            HT[r * K:(r + 1) * K].copy_(Hn.t())
            W[r * K:(r + 1) * K].copy_(Wn)


def init_factors(X: torch.Tensor, K: int, seeds, init: str = "random", comm=None,
                 row_offset: int = 0):
    """Initial (HT (R*K x N_loc), W (R*K x G)) for a single-K replicate batch."""
    R = len(seeds)
    N, G = X.shape
    HT = torch.empty((R * K, N), device=X.device, dtype=X.dtype)
    W = torch.empty((R * K, G), device=X.device, dtype=X.dtype)
    init_into(HT, W, X, K, seeds, init, comm, row_offset)
    return HT, W


# =============================================================================== state
def _to_device(a: np.ndarray, dev: torch.device) -> torch.Tensor:
    """int64 host index array -> device, without a synchronising pageable copy."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64))
    if dev.type == "cuda":
        return t.pin_memory().to(dev, non_blocking=True)
    return t


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
        idx = _to_device(inv, dev)
        # one packed device->host copy instead of eight small synchronising ones
        keys = ("err", "n_pass", "converged")
        rows5 = torch.stack([self.state[k][idx].to(torch.float64) for k in keys] +
                            [self.h_iters[idx].to(torch.float64),
                             self.w_iters[idx].to(torch.float64)])
        flat = torch.cat([rows5.view(-1)] + [t.view(-1)[:1].to(torch.float64) for t in extra]) \
            if len(extra) else rows5.view(-1)
        flat = flat.cpu().numpy()
        m = idx.numel()
        packed, ext = flat[:5 * m].reshape(5, m), flat[5 * m:]
        return (HT, W, self.kpos[inv], packed[0], packed[1].astype(np.int64), packed[2] != 0,
                packed[3].astype(np.int64), packed[4].astype(np.int64), ext)


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
        self.pending = None   # (event, host_flags, n)

    def _frac(self, n: int) -> float:
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
        flags = torch.empty(n, dtype=torch.int32, pin_memory=True)
        # (a flag copy on a side stream removed the ~5 us gap per pass in the trace but was
        # slower end to end -- headline -2 %, K grid -5.5 %, profiles/r3y_*: the stream
        # switch and event sit on the host's enqueue path)
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
                 dtype=torch.float32):
        self.uid = next(_FEED_UIDS)
        self.seeds = np.asarray(seeds, dtype=np.int64)
        self.ks = np.asarray(ks, dtype=np.int64)
        R = self.seeds.size
        self.offs = np.concatenate([[0], np.cumsum(self.ks)[:-1]]).astype(np.int64)
        self.queue = {int(K): collections.deque(np.flatnonzero(self.ks == K).tolist())
                      for K in np.unique(self.ks)}
        tot = int(self.ks.sum())
        self.store = {
            "offs": torch.from_numpy(self.offs).to(dev),
            "W": torch.empty((tot, G), device=dev, dtype=dtype),
            "HT": torch.empty((tot, N), device=dev, dtype=dtype) if keep_usages else None,
            # err_init, err_prev, err | active, converged, n_pass, h_iters, w_iters
            "sf": torch.zeros((3, R), dtype=torch.float64, device=dev),
            "si": torch.zeros((5, R), dtype=torch.int32, device=dev),
        }
        self.R = R
        self.rings: dict = {}     # K -> ring (see NMFBatchSolver._stream_ring)
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


_SQ_NORM_CACHE: dict = {}


def _sq_norm(X: torch.Tensor, rows: int = 1 << 16) -> float:
    """||X||_F^2 accumulated in float64 over row blocks (no full float64 copy of X:
    a 10M x 5k matrix would need 400 GB).  Memoised per tensor storage and version
    (factorize builds one solver per K over the same resident X); an in-place
    modification of X bumps its version and invalidates the entry, and a weak reference
    guards against a new tensor reusing a freed address."""
    key = (id(X), X.data_ptr(), tuple(X.shape), tuple(X.stride()), X.dtype, X._version)
    hit = _SQ_NORM_CACHE.get(key)
    if hit is not None and hit[0]() is X:      # same live tensor object, same contents
        return hit[1]
    tot = torch.zeros((), dtype=torch.float64, device=X.device)
    for a in range(0, X.shape[0], rows):
        xb = X[a:a + rows]
        tot += torch.linalg.vector_norm(xb, dtype=torch.float64).square()
    val = float(tot)
    if len(_SQ_NORM_CACHE) > 16:
        _SQ_NORM_CACHE.clear()
    _SQ_NORM_CACHE[key] = (weakref.ref(X), val)
    return val


def _inner_solve(algo: str, x3: torch.Tensor, numer3: torch.Tensor, gram3: torch.Tensor,
                 **kw) -> None:
    """One half-step on x3 (R, K, n) in place.  'mu' / 'hals' run the fused iterative
    kernels (ops.solve); 'bpp' solves every column's NNLS exactly (models/bpp.py) and
    fills the same optional outputs: lin/quad (trace-trick loss terms) and iters."""
    if algo != "bpp":
        ops.solve("hals" if algo == "halsvar" else algo, x3, numer3, gram3, **kw)
        return
    gram_of = kw.pop("gram_of", None)
    if gram3 is None:
        gram3 = ops.gram(gram_of)
    planes, colmul = kw.pop("planes", None), kw.pop("planes_colmul", None)
    R, K = x3.shape[0], x3.shape[1]
    active = kw.get("active")
    live = None if active is None else (active[:R] != 0)
    g, b = gram3, numer3
    if live is not None:
        # finished replicates' statistics are stale (possibly never written): give them a
        # trivial, finite system; their result is discarded below
        keep = live.view(R, 1, 1)
        g = torch.where(keep, gram3, torch.eye(K, dtype=gram3.dtype, device=gram3.device))
        b = torch.where(keep, numer3, torch.zeros((), dtype=numer3.dtype, device=numer3.device))
    xn = nnls_bpp(g, b, l1=kw.get("l1_den", 0.0), l2=kw.get("l2", 0.0))
    x3.copy_(xn if live is None else torch.where(live.view(R, 1, 1), xn, x3))
    lin_out, quad_out = kw.get("lin_out"), kw.get("quad_out")
    if lin_out is not None or quad_out is not None:
        lin, quad = bpp_objective_terms(x3, numer3, gram3)
        for out, v in ((lin_out, lin), (quad_out, quad)):
            if out is not None:
                v = v.to(out.dtype)
                out[:R] = v if live is None else torch.where(live, v, out[:R])
    iters = kw.get("iters_out")
    if iters is not None:
        iters[:R] += 1 if live is None else live.to(iters.dtype)
    if planes is not None:   # bpp: the same planes epilogue, as a separate split
        ops.split_planes(x3.reshape(R * K, x3.shape[2]), planes, col_mul=colmul)


class RowBlocks:
    """A cells x genes float32 matrix that is never whole on the device: ``blocks()``
    yields (row_start, (rows, G) float32 device block) over all rows, in order, and may be
    called several times (each call regenerates or re-reads the blocks).  Row starts must
    be multiples of 4 (the split planes' k offsets).  ``RowBlocks.of(X)`` views a resident
    tensor the same way."""

    def __init__(self, n_rows: int, n_cols: int, blocks_fn, device):
        self.shape = (int(n_rows), int(n_cols))
        self.device = torch.device(device)
        self.dtype = torch.float32
        self._fn = blocks_fn

    def blocks(self):
        for a, blk in self._fn():
            if a % 4:
                raise ValueError(f"RowBlocks: block start {a} is not a multiple of 4")
            yield a, blk

    @classmethod
    def of(cls, X: torch.Tensor, rows: int = 1 << 16) -> "RowBlocks":
        N, G = X.shape
        return cls(N, G, lambda: ((a, X[a:a + rows]) for a in range(0, N, rows)), X.device)


def _block_colstats(src: RowBlocks):
    """(min positive, float64 sum of squares, any-negative, float64 sum) per column over
    every block (ops.colstats per block, combined)."""
    N, G = src.shape
    dev = src.device
    mn = torch.full((G,), float("inf"), dtype=torch.float32, device=dev)
    sq = torch.zeros(G, dtype=torch.float64, device=dev)
    sm = torch.zeros(G, dtype=torch.float64, device=dev)
    neg = torch.zeros(G, dtype=torch.int32, device=dev)
    for _, blk in src.blocks():
        m_, q_, n_ = ops.colstats(blk)
        torch.minimum(mn, m_, out=mn)
        sq += q_
        neg |= n_.to(torch.int32)
        sm += blk.sum(dim=0, dtype=torch.float64)
    return mn, sq, neg, sm


def _count_units(X, stats=None):
    """Per-gene unit u (G,) with X == C * u for a non-negative INTEGER matrix C, or None.

    cNMF's normalised counts are raw counts over a per-gene std (cnmf.py:670-681), so the
    unit of column g is (count 1) / std_g: the smallest positive entry m of the column
    over its smallest count d.  d is tried as 1..8 (one fused pass, ops.count_unit_check),
    then -- highly expressed genes whose every count exceeds 8 -- as round(m / gap) with
    gap the smallest difference between distinct entries; a column of zeros gets u = 1.
    Accepted only if every entry of every column is an integer multiple of its unit to
    fp32 rounding (|X/u - round(X/u)| <= 4e-7 * X/u + 1e-4) and C < 65536.  ``stats``:
    the (min_pos, sumsq, neg) of ops.colstats when already computed.  ``X`` may be a
    :class:`RowBlocks` (the check then runs block by block)."""
    N, G = X.shape
    if N == 0:
        return None
    src = X if isinstance(X, RowBlocks) else None
    if stats is not None:
        mn_t, _, neg = stats[:3]
    elif src is not None:
        mn_t, _, neg, _ = _block_colstats(src)
    else:
        mn_t, _, neg = ops.colstats(X)
    if src is None:
        bad_t = ops.count_unit_check(X, mn_t)     # skips empty columns (min_pos = inf)
    else:
        bad_t = torch.zeros(G, dtype=torch.int32, device=src.device)
        for _, blk in src.blocks():
            bad_t |= ops.count_unit_check(blk, mn_t)
    # one host round trip for the per-gene decisions
    host = torch.stack([mn_t.double(), bad_t.double(), neg.double()]).cpu().numpy()
    mn, bad, neg_h = host[0], host[1].astype(np.int64), host[2] != 0
    empty = ~np.isfinite(mn)
    mn = np.where(empty, 1.0, mn)
    if neg_h.any():
        return None
    inv = (~bad) & 0xFF                         # bit d-1 set: d works
    d = np.zeros(G, dtype=np.int64)
    for k in range(8, 0, -1):
        d = np.where((inv >> (k - 1)) & 1, k, d)
    unit = np.where(d > 0, mn / np.maximum(d, 1), np.nan)
    unit[empty] = 1.0
    todo = np.flatnonzero(np.isnan(unit))
    if todo.size > 64:
        return None
    if todo.size and src is not None:     # the few columns the gap rule needs, gathered
        tt = torch.as_tensor(todo, device=src.device)
        cols = torch.cat([blk.index_select(1, tt) for _, blk in src.blocks()])
        colmap = {g: cols[:, i] for i, g in enumerate(todo.tolist())}
    else:
        colmap = None
    for g in todo.tolist():
        xg = colmap[g] if colmap is not None else X[:, g]
        v = torch.unique(xg)
        v = v[v > 0]
        dv = torch.diff(v)
        if dv.numel() == 0:
            return None
        u = float(mn[g]) / max(1.0, round(float(mn[g]) / float(dv.min())))
        c = xg / u
        if bool((((c - torch.round(c)).abs() > 4e-7 * c + 1e-4) | (c >= 65535.5)).any()):
            return None
        unit[g] = u
    # mn / d in float32 arithmetic, as the device check evaluated it
    return torch.from_numpy((mn.astype(np.float32) / np.maximum(d, 1).astype(np.float32))
                            .astype(np.float32) if todo.size == 0 else unit.astype(np.float32)
                            ).to(mn_t.device).contiguous()


class _XPlanes:
    """Exact bf16 planes of the data matrix for the split-precision GEMMs
    (ops.gemm_planes), built once per solver: ``x`` (pb, N+pad, Gp) with genes on k (the
    H-side numerator W X_c^T) and ``xt`` (pb, G, Np) with cells on k (the statistics
    H_c^T X_c).  Integer data (cNMF norm counts) is stored as its count matrix C in one
    bf16 plane (C <= 256) or two (C < 65536) with the per-gene ``unit`` folded into the
    other operand / the output columns; other data as three planes of X itself."""

    def __init__(self, X, stats=None):
        """``X``: the resident fp32 matrix, or a :class:`RowBlocks` (planes built block by
        block; no full fp32 copy is ever made -- nor is one needed for a resident X: the
        count matrix is rounded per block)."""
        N, G = X.shape
        self.N, self.G = N, G
        src = X if isinstance(X, RowBlocks) else RowBlocks.of(X)
        dev = src.device
        unit = _count_units(X, stats)
        if unit is not None:
            cmax = 0.0
            for _, blk in src.blocks():
                if blk.numel():
                    cmax = max(cmax, float(torch.round(blk / unit).max()))
            # integers 0..256 are exact in one bf16 plane, 0..65535 in two (hi + the
            # exact residual): the split below is lossless by construction
            self.pb = 1 if cmax <= 256 else 2
            if cmax >= 65536:
                unit, self.pb = None, self._float_planes(G)
        else:
            self.pb = self._float_planes(G)
        self.unit = unit
        self.Gp = -(-G // 64) * 64
        self.Np = -(-N // 64) * 64 + 64
        self.x = torch.zeros((self.pb, N + 128, self.Gp), dtype=torch.int16, device=dev)
        self.xt = torch.zeros((self.pb, G, self.Np), dtype=torch.int16, device=dev)
        for a, blk in src.blocks():
            n = blk.shape[0]
            C = torch.round(blk / unit) if unit is not None else blk
            ops.split_planes(C, self.x[:, a:a + n])
            Ct = C.t().contiguous()                               # (G, cells of the block)
            ops.split_planes(Ct, self.xt[:, :, a:a + -(-n // 4) * 4])
            del C, Ct

    @staticmethod
    def bytes_needed(N: int, G: int, pb: int) -> int:
        """Device bytes of the two plane layouts for ``pb`` planes."""
        return 2 * pb * ((N + 128) * (-(-G // 64) * 64) + G * (-(-N // 64) * 64 + 64))

    @staticmethod
    def _float_planes(G: int) -> int:
        """B planes of non-count data: 2 (hi + mid, <= 2^-16 relative per element, the
        same bound the engine accepts for the A operand, ops.gemm_a_planes) once the
        numerator's reduction runs over >= 1024 genes -- inside the fp32 GEMM's own error
        there (test_gemm_two_b_planes_within_fp32_library_error); else 3 (exact).  Two
        planes make a product 4 MFMAs instead of 5 (2 for counts) and halve nothing else."""
        return 3 if G < 1024 else 2

    @staticmethod
    def build(X: torch.Tensor, stats=None, reserve: int = 0):
        """Planes for X when the split GEMM path applies (GPU, fp32, memory), else None.
        ``reserve``: device bytes the caller still has to allocate after the planes (the
        fused step's slabs, plane buffers and statistics), kept free so a run that does
        not fit takes the documented fp32 fallback here instead of failing partway."""
        if X.device.type != "cuda" or X.dtype != torch.float32 or \
                os.environ.get("CNMF_GEMM", "planes") != "planes":
            return None
        N, G = X.shape
        # sized by the most planes the data can take (2 for counts above 256, 2 or 3 for
        # non-count data: _float_planes) plus one row block's temporaries -- not 3 planes
        # + a full fp32 copy of X as before (that refused 10M x 5k on one GPU)
        pb = max(2, _XPlanes._float_planes(G))
        need = _XPlanes.bytes_needed(N, G, pb) + 3 * 4 * min(N, 1 << 16) * G + int(reserve)
        free, _ = torch.cuda.mem_get_info(X.device)
        if need > 0.9 * free:
            _warn_once(f"split-precision GEMM planes need {need / 1e9:.1f} GB, "
                       f"{free / 1e9:.1f} GB free: the data-side GEMMs fall back to the fp32 "
                       "library GEMM (pass the matrix as nmf.PlanesOnlyX to hold it as "
                       "planes only)")
            return None
        return _XPlanes(X, stats)


_WARNED: set = set()


def _warn_once(msg: str) -> None:
    if msg not in _WARNED:
        _WARNED.add(msg)
        import warnings

        warnings.warn(msg, RuntimeWarning, stacklevel=3)


class PlanesOnlyX:
    """A cells x genes matrix held on the device ONLY as the split-GEMM planes (plus its
    statistics), built block by block from a :class:`RowBlocks` source: the fp32 matrix is
    never resident.  At 10M cells x 5k genes the fp32 matrix alone is 200 GB and its
    count planes 100-200 GB, which do not fit one 288 GB MI355X together
    (tools/bench_large.py --planes-only).  ``NMFBatchSolver`` takes it in place of X for
    online Frobenius MU/HALS with random init -- every other use of X raises."""

    def __init__(self, src: RowBlocks):
        self.shape, self.device, self.dtype = src.shape, src.device, torch.float32
        mn, sq, neg, sm = _block_colstats(src)
        self.x_sq = float(sq.sum())
        self.sum = float(sm.sum())
        self.planes = _XPlanes(src, stats=(mn, sq, neg))


def kernel_max_rank(beta: float, algo: str) -> int | None:
    """Largest K the native kernels factorise (None: no limit -- 'bpp' solves its NNLS
    blocks with torch linear algebra): Frobenius MU 128 (padded, native_rank), HALS /
    halsvar 64, KL 64 and the other beta-divergences 56 (padded to a multiple of 8 above
    32; beta_planes_wide*.hip -- an IS / general-beta K = 64 panel pair exceeds the LDS).
    Larger ranks are routed to the eager PyTorch ops on the same GPU (NMFBatchSolver.run,
    logged)."""
    if algo == "bpp":
        return None
    if beta != 2.0:
        return 64 if beta == 1.0 else 56
    return 128 if algo == "mu" else 64


def native_rank(K: int) -> int:
    """The rank the GPU kernels run a rank-K replicate at: K itself for K <= 32, else K
    padded with zero components to a multiple of 8 (<= 64) or of 16 (<= 128, MU only: the
    matrix-core wide solve, solve_wmfma.hip) -- a zero row of W / H stays zero under MU
    (rate 0 where the denominator vanishes) and HALS (zero diagonal), and contributes
    nothing to the Gram matrices or the loss, so the padded solve IS the rank-K solve
    (cnmf.py:1416 takes any -k)."""
    K = int(K)
    if K <= 32:
        return K
    if K <= 64:
        return -(-K // 8) * 8
    if K > 128:
        raise ValueError(f"K={K}: the native kernels cover K <= 128")
    return -(-K // 16) * 16


# first pass of a recurring batch layout from its captured graph (not eager) -- removes
# the ~330 us of host-paced idle of the compaction pass (profiles/r3y_passes.txt)
_LAYOUT_REPLAY = True
# fused step: split-K GEMMs of up to this many k slices hand their raw slabs to the
# consuming solve; deeper splits (the few-replicate tail) are reduced by the GEMM's own
# pass -- the solve would read every slab per element
_FUSED_MAX_SLABS = 4


def _graphs_enabled(X: torch.Tensor) -> bool:
    """Capture repeated passes into HIP graphs (GPU only, opt-in: CNMF_GRAPHS=1).  Off by
    default: a compaction changes the layout every few passes, and re-capturing cost more
    than the launches it saved on the bench shape (27.2 vs 20.5 ms per 100 replicates)."""
    return X.device.type == "cuda" and os.environ.get("CNMF_GRAPHS", "0") == "1"


def _chunks(n_rows: int, c: int, n_steps: int):
    out = []
    for s in range(n_steps):
        a = min(s * c, n_rows)
        b = min(a + c, n_rows)
        out.append((a, b))
    return out


class NMFBatchSolver:
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
        feed = _Feed(seeds, ks, dev, N, G, keep_usages, self.X.dtype)
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
        # reads and writes); graphs follow the usual rule
        arena = self._arena(kpos)
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
        feed.ctr = torch.zeros(1 + len(st.groups), dtype=torch.int32, device=dev)
        feed.seq = torch.zeros(1, dtype=torch.int32, device=dev)
        feed.box = ops.HostMailbox(1 + len(st.groups))
        for i, g in enumerate(st.groups):
            feed.occ[g.K] = torch.from_numpy(first[g.p0:g.p0 + g.n].astype(np.int32)).to(dev)
            feed.plan[g.K] = torch.empty(2 * g.n, dtype=torch.int32, device=dev)
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
        HTo = store["HT"] if store["HT"] is not None else torch.empty((0, N), device=dev)
        return NMFResult(HT=HTo, W=store["W"], err=err, n_iter=rest[1].astype(np.int64),
                         converged=rest[0] != 0, seeds=seeds,
                         K=int(uni[0]) if uni.size == 1 else None, stats=stats, ks=ks)

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
        buf = self._ws.get(key)
        if buf is None or buf.shape[1] < rows or buf.shape[2] != cols:
            buf = torch.zeros((3, rows, cols), dtype=torch.int16, device=self.X.device)
            self._ws[key] = buf
        return buf

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
            torch.cuda.set_device(dev)
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

    # ------------------------------------------------------------------ graphs / arena
    def _graphs_wanted(self, kpos) -> bool:
        """Replay the fused online passes from HIP graphs captured once per batch layout
        and kept across runs (CNMF_GRAPHS: 'auto' (default) = batches of <= 256
        replicates, whose passes are short enough for the host's per-pass enqueue to
        show; '1' any batch; '0' never).  Needs the fused step's preconditions (checked
        again per run by _fused_ok)."""
        env = os.environ.get("CNMF_GRAPHS", "auto")
        o = self.opts
        if env == "0" or self.X.device.type != "cuda" or self.beta != 2.0 or o.mode != "online":
            return False
        if env != "1" and len(kpos) > 256:
            return False
        return (o.algo == "mu" and o.online_stats == "pass" and o.online_inner_conv == "loss"
                and not self.comm.is_distributed and int(np.max(kpos)) <= 64
                and os.environ.get("CNMF_FUSED_STEP", "1") != "0"
                and all(v == 0.0 for v in (o.l1_H, o.l2_H, o.l1_W, o.l2_W)))

    def _arena(self, kpos) -> dict:
        """HT / W / state tensors of a batch with this rank vector, kept across runs on the
        current stream (see _Batch's arena)."""
        import collections

        key = (tuple(int(k) for k in kpos), ops._stream_ptr(self.X))
        if not hasattr(self, "_arenas"):
            self._arenas = collections.OrderedDict()
        a = self._arenas.get(key)
        if a is None:
            N, G = self.X.shape
            dev, tot, R = self.X.device, int(np.sum(kpos)), len(kpos)
            sf = torch.zeros((3, R), dtype=torch.float64, device=dev)
            si = torch.zeros((5, R), dtype=torch.int32, device=dev)
            a = {"HT": torch.zeros((tot, N), device=dev, dtype=self.X.dtype),
                 "W": torch.zeros((tot, G), device=dev, dtype=self.X.dtype),
                 "sf": sf, "si": si,
                 "state": {"err_init": sf[0], "err_prev": sf[1], "err": sf[2],
                           "active": si[0], "converged": si[1], "n_pass": si[2]},
                 "h_iters": si[3], "w_iters": si[4],
                 "gate": torch.ones(1, dtype=torch.int32, device=dev),
                 "slots": collections.OrderedDict()}
            self._arenas[key] = a
            while len(self._arenas) > 4:
                self._arenas.popitem(last=False)
        else:
            self._arenas.move_to_end(key)
        return a

    def _slot(self, st: _Batch, steps) -> dict:
        """Per-layout slot of an arena batch: the fused step's workspaces (fixed addresses),
        a capture stream and, once captured, the pass's HIP graph."""
        a = st.arena
        # (a streaming run's pass graph holds its feed's ring / store addresses)
        key = (st.n_act, tuple(int(k) for k in st.kpos[:st.n_act]),
               tuple(tuple(b) for b in steps), st.feed.uid if st.feed is not None else None)
        slots = a["slots"]
        sl = slots.get(key)
        if sl is None:
            sl = {"fb": self._fused_bufs(st, steps), "graph": None, "failed": False,
                  "stream": torch.cuda.Stream(self.X.device)}
            slots[key] = sl
            while len(slots) > 24:
                slots.popitem(last=False)
        else:
            slots.move_to_end(key)
        return sl

    def _replay_slot(self, sl: dict, st: _Batch, steps) -> bool:
        """Run one non-final fused pass from the slot's graph (captured on first use, on
        the slot's own stream, from a pass whose operands are already in place).  False:
        capture unavailable -- the caller runs the pass eagerly."""
        if sl["failed"]:
            return False
        if sl["graph"] is None:
            g = torch.cuda.CUDAGraph()
            main = torch.cuda.current_stream(self.X.device)
            o = self.opts
            ops.coop_reserve(self.X.device, sl["stream"].cuda_stream,
                             max(gr.n for gr in st.groups), int(o.online_chunk_max_iter),
                             int(o.inner_check_every))
            sl["stream"].wait_stream(main)
            try:
                with torch.cuda.stream(sl["stream"]):
                    g.capture_begin()
                    try:
                        self._fused_pass(st, steps, sl["fb"], False)
                    finally:
                        g.capture_end()
            except RuntimeError as e:
                sl["failed"] = True
                sl["error"] = str(e)
                log.warning("pass graph capture failed (%s); eager passes for this layout", e)
                return False
            main.wait_stream(sl["stream"])
            sl["graph"] = g
        sl["graph"].replay()
        return True

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
            # the reduce-scattered W-solve partitions the replicates of ONE rank group
            # (mixed-K DP batches take the unfused, all-reduced step)
            if (len(st.groups) != 1 or os.environ.get("CNMF_DP_FUSED", "1") == "0"
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

    # ------------------------------------------------------------------ DP fused step
    def _fused_bufs_dp(self, st: _Batch, steps) -> dict:
        """Workspaces of the cell-sharded fused step (_fused_pass_dp).  The replicates are
        partitioned into ``world`` equal position chunks of Rr (the last rank's chunk may
        hold fewer real ones); every exchanged buffer is padded to world * Rr positions so
        each rank's chunk is one contiguous block for reduce-scatter / all-gather."""
        comm = self.comm
        xp = self._planes()
        dev = self.X.device
        G = self.X.shape[1]
        (g,) = st.groups
        K, R, world, me = g.K, g.n, comm.world_size, comm.rank
        Rr = -(-R // world)
        Rp = Rr * world
        own0, own1 = min(R, me * Rr), min(R, (me + 1) * Rr)
        cws = [b - a for (a, b), in steps]
        bk = ops.planes_bk(xp.pb)
        kd_max = max(-(-cw // bk) * bk for cw in cws)
        ks_n = max(ops.gemm_plan(R * K, cw, xp.Gp, xp.pb)[1] for cw in cws)
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
        # ONE reduce-scatter per online step: rank r's chunk is [dB rows of its replicates
        # | their per-slice partial H^T H], and ONE all-gather: rank r's chunk is [the
        # spectra bf16 planes of its replicates | their W W^T partials | lin | quad] as
        # bytes -- the W-solve writes its outputs straight into that chunk
        n_db, n_hh = Rr * K * G, Rr * S_h * K * K
        pl_b, ww_b = wpl_n * Rr * K * xp.Gp * 2, Rr * S_w * K * K * 4
        n_ag = pl_b + ww_b + 8 * Rr
        rs_own = torch.empty(n_db + n_hh, **f32)
        ag_own = torch.zeros(n_ag, device=dev, dtype=torch.uint8)
        fb = {
            "K": K, "R": R, "Rr": Rr, "Rp": Rp, "own": (own0, own1), "S_h": S_h, "S_w": S_w,
            "wpl_n": wpl_n,
            "wpl": torch.zeros((3, Rp * K, xp.Gp), device=dev, dtype=torch.int16),
            "hpl": torch.zeros((3, R * K, kd_max), device=dev, dtype=torch.int16),
            "slabN": torch.empty(ks_n * R * K * max(cws), **f32),
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
            "prepped": None,
        }
        return fb

    @staticmethod
    def _dp_pack_rs(fb: dict) -> None:
        """[dB | HHp] of every replicate into the reduce-scatter buffer, rank-chunked."""
        world, Rr, K = fb["rs"].shape[0], fb["Rr"], fb["K"]
        n_db = fb["dB_own"].numel()
        rs = fb["rs"]
        rs[:, :n_db].copy_(fb["dB"].view(world, n_db))
        rs[:, n_db:].copy_(fb["HHp"].view(world, -1))

    @staticmethod
    def _dp_unpack_ag(fb: dict, last: bool) -> None:
        """Every rank's chunk of the all-gather into the full-batch planes, W W^T partials
        and (last step) lin / quad."""
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

    def _fused_pass_dp(self, st: _Batch, steps, fb: dict, final: bool) -> None:
        """One online pass of the fused step on a cell shard (SURVEY.md §2.5c / §2.6 item
        1).  Per online step every rank runs the numerator GEMM and the pipelined H-solve
        on its cells of the global chunk and the statistics GEMM dB = H_loc^T X_loc; then
        ONE reduce-scatter of the packed [dB | partial H^T H] hands each rank the
        rank-summed statistics of ITS replicate chunk, the rank W-solves only those (1/world
        of the spectra work) straight into its chunk of ONE all-gather of [bf16 spectra
        planes | per-slice W W^T partials | lin | quad] -- two collectives per step (five
        before the packing: dB, HHp, WWp and one per plane, +2 on the last step), the bytes
        of one all-reduce of dB, the W-solve no longer replicated on every rank (the
        unfused DP step all-reduces [dB | dA] and re-solves every replicate everywhere).
        Same updates and stopping rules as the single-GPU fused step; rank-summed
        statistics in RCCL's order."""
        o = self.opts
        comm = self.comm
        xp = self._planes()
        X = self.X
        G = X.shape[1]
        HT, W = st.views()
        (g,) = st.groups
        K, R, Rr, Rp = fb["K"], fb["R"], fb["Rr"], fb["Rp"]
        own0, own1 = fb["own"]
        n_own = own1 - own0
        S_h, S_w = fb["S_h"], fb["S_w"]
        active = st.active_mask()
        n = st.n_act
        h_it, w_it = st.h_iters[:n], st.w_iters[:n]
        bk = ops.planes_bk(xp.pb)
        rows = R * K
        wpl, hpl_all = fb["wpl"], fb["hpl"]
        if fb["prepped"] != st.uid:
            # W is replicated at the start of a run: every rank forms every Gram / plane
            fb["WWp"].zero_()
            fb["WWp"][:R, 0].copy_(ops.gram(g.rep3(W)))
            ops.split_planes(W, wpl[:, :rows], col_mul=xp.unit)
            fb["wwp_n"] = 1
            fb["prepped"] = st.uid
        unit = xp.unit
        wpl_n = ops.gemm_a_planes(xp.Gp)
        o0, o1 = own0 * K, own1 * K
        Wown = W[o0:o1].view(n_own, K, G) if n_own else None
        last_s = len(steps) - 1
        for s_, ((a, b),) in enumerate(steps):
            cw = b - a
            last = s_ == last_s
            ks_n = ops.gemm_planes(None, wpl[:wpl_n, :rows], xp.x[:, a:], rows, cw, xp.Gp,
                                   raw_slab=fb["slabN"], raw_max=_FUSED_MAX_SLABS)
            kd = -(-cw // bk) * bk
            hpl = hpl_all[:, :, :kd]
            hpl_n = ops.gemm_a_planes(kd)
            if cw > 0:
                numer = fb["slabN"].as_strided((R, K, cw), (K * cw, cw, 1), 0)
                ops.solve("mu", g.rep3(HT[:, a:b]), numer, None,
                          max_iter=o.online_chunk_max_iter, tol=o.online_h_tol, eps=o.eps,
                          iters_out=h_it, conv_mode=1, check_every=o.inner_check_every,
                          active=active, planes=hpl, planes_n=hpl_n, numer_slabs=ks_n,
                          numer_slab_stride=rows * cw, coop=S_h,
                          gram_parts=fb["WWp"][:R], gram_parts_n=fb["wwp_n"],
                          gram_parts_out=fb["HHp"][:R], coop_device_gen=True)
                ops.gemm_planes(fb["dB"], hpl[:hpl_n], xp.xt[:, :, a:], rows, G, kd)
            else:      # no cells of this chunk here: zero contributions
                fb["dB"][:rows].zero_()
                fb["HHp"][:R].zero_()
            self._dp_pack_rs(fb)
            comm.reduce_scatter_(fb["rs_own"], fb["rs"])
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
                    conv_mode=1, check_every=o.inner_check_every, active=active[own0:own1],
                    planes=fb["ag_pl"][:, :n_own * K], planes_colmul=unit, planes_n=wpl_n,
                    numer_scale=unit,
                    numer_base=None if s_ == 0 else fb["B_own"][:n_own * K].view(n_own, K, G),
                    numer_out=None if last else fb["B_own"][:n_own * K].view(n_own, K, G),
                    gram_parts=fb["HHp_own"][:n_own], gram_parts_n=S_h,
                    gram_out=None if last else A_out[:n_own],
                    gram_parts_out=wwp[:n_own], coop=S_w, coop_device_gen=True)
            fb["wwp_n"] = S_w
            comm.all_gather_into_(fb["ag"], fb["ag_own"])
            self._dp_unpack_ag(fb, last)
        ops.conv_update(fb["lin"], fb["quad"], self.x_sq, {k: v[:n] for k, v in st.state.items()},
                        n, -1, o.tol, final=final, gate=st.gate,
                        max_pass=int(o.online_max_pass))

    def _dp_gather_w(self, st: _Batch, fb: dict) -> None:
        """End of a DP fused run: every rank's W-solved spectra rows to every rank."""
        _, W = st.views()
        K, R, Rr, Rp = fb["K"], fb["R"], fb["Rr"], fb["Rp"]
        G = W.shape[1]
        me = self.comm.rank
        Wp = torch.zeros((Rp * K, G), device=W.device, dtype=W.dtype)
        o0, o1 = me * Rr * K, min(R, (me + 1) * Rr) * K
        if o1 > o0:
            Wp[o0:o1].copy_(W[o0:o1])
        self.comm.all_gather_into_(Wp, Wp[me * Rr * K:(me + 1) * Rr * K])
        W.copy_(Wp[:R * K])
        it = torch.zeros(Rp, dtype=torch.int32, device=W.device)   # W-solve sweep counts
        o0, o1 = me * Rr, min(R, (me + 1) * Rr)
        if o1 > o0:
            it[o0:o1].copy_(st.w_iters[o0:o1])
        self.comm.all_gather_into_(it, it[me * Rr:(me + 1) * Rr])
        st.w_iters[:R].copy_(it[:R])

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
        feed.ctr = torch.cat([feed.ctr[:1]] + [
            feed.ctr.new_full((1,), feed.rings[g.K]["published"]) for g in st.groups])
        for g in st.groups:
            feed.occ[g.K] = occ_new[g.p0:g.p0 + g.n].clone()
            feed.plan[g.K] = torch.empty(2 * g.n, dtype=torch.int32, device=dev)
            ring = feed.rings[g.K]
            ring["head"] = feed.ctr[1 + st.groups.index(g):2 + st.groups.index(g)]

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

    def _enqueue_fused(self, st: _Batch, steps, cur: dict) -> None:
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
                        max_pass=int(o.online_max_pass))
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
                        with torch.cuda.graph(graph):
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

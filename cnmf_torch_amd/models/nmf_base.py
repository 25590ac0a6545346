"""Options, results, initialisation, rank routing and the X operands of the NMF engine
(split out of models/nmf.py; see that module's docstring for the algorithms)."""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch
from torch.utils.weak import WeakIdKeyDictionary

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
        # planes built ahead for this tensor: handed over once (the solver owns them
        # from here and frees them with itself; nothing keeps a second copy alive)
        ahead = _PLANES_AHEAD.pop(X, None) if isinstance(X, torch.Tensor) else None
        if ahead is not None and ahead[0] == (X.data_ptr(), X._version):
            # allocated on the background builder's (pooled) stream and used from here on
            # on this one: without record_stream their blocks would return to the builder
            # stream's pool at free while this stream's kernels may still read them
            cur = torch.cuda.current_stream(X.device)
            for v in vars(ahead[1]).values():
                for t in (v if isinstance(v, (list, tuple)) else (v,)):
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        t.record_stream(cur)
            return ahead[1]
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



# planes built ahead of the solver for a resident X (cNMF.prepare's background thread,
# planes_ahead), keyed by the tensor's identity and valid while its storage and version
# are unchanged
_PLANES_AHEAD = WeakIdKeyDictionary()


def planes_ahead(X: torch.Tensor) -> None:
    """Build and keep ``X``'s split-GEMM planes now, for the solver that will factorise
    this same resident tensor (factorize after prepare in one process): the unit check,
    two host round trips and the plane split leave factorize's critical path.  Only when
    they take under a quarter of the free device memory (no workspace reserve is known
    yet)."""
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda" or X.dtype != torch.float32:
        return
    free, _ = torch.cuda.mem_get_info(X.device)
    if _XPlanes.bytes_needed(X.shape[0], X.shape[1], 2) > 0.25 * free:
        return
    xp = _XPlanes.build(X)
    if xp is not None:
        _PLANES_AHEAD[X] = ((X.data_ptr(), X._version), xp)


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
    """Largest K the native kernels factorise (None: no limit).  Frobenius MU: any K --
    register-tiled kernels up to 128 (padded, native_rank), the rank-general solve beyond
    (solve_any.hip: library Gram-x GEMM + HIP update / objective / stop kernels); HALS /
    halsvar: 512 (64 on the tiled kernels, solve_any.hip's LDS-resident Gauss-Seidel sweep
    above); the beta-divergences: any K (split-bf16 panel kernels to KL 64 / IS 56, the
    rank-general path beyond: library GEMMs for P and the contractions, beta_any.hip for
    the terms); 'bpp' solves its NNLS blocks with torch linear algebra.  Larger ranks are
    routed to the eager PyTorch ops on the same GPU (NMFBatchSolver.run, logged)."""
    if algo == "bpp" or beta != 2.0:
        return None
    return None if algo == "mu" else 512


def native_rank(K: int) -> int:
    """The rank the GPU kernels run a rank-K replicate at: K itself for K <= 32, else K
    padded with zero components to a multiple of 8 (<= 64) or of 16 (<= 128: MU's
    matrix-core wide solve, solve_wmfma.hip), and K itself above 128 (the rank-general
    solve, solve_any.hip) -- a zero row of W / H stays zero under MU
    (rate 0 where the denominator vanishes) and HALS (zero diagonal), and contributes
    nothing to the Gram matrices or the loss, so the padded solve IS the rank-K solve
    (cnmf.py:1416 takes any -k)."""
    K = int(K)
    if K <= 32:
        return K
    if K <= 64:
        return -(-K // 8) * 8
    if K > 128:
        return K        # the rank-general solve (solve_any.hip) takes K as it is
    return -(-K // 16) * 16



# first pass of a recurring batch layout from its captured graph (not eager) -- removes
# the ~330 us of host-paced idle of the compaction pass (profiles/r3y_passes.txt)
_LAYOUT_REPLAY = True


# fused step: split-K GEMMs of up to this many k slices hand their raw slabs to the
# consuming solve; deeper splits (the few-replicate tail) are reduced by the GEMM's own
# pass -- the solve would read every slab per element
# (re-measured in round 6 with the swap compaction: caps 4 / 8 / 16 gave 13,930-14,010 /
# 13,774-13,872 / 13,369-13,373 rep/s, profiles/r6k_*)
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

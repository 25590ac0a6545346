"""Harmony batch correction on the device (C30, C37; preprocess.py:9-18, 342-388).

The reference calls ``harmonypy.run_harmony`` (not installed here) and then applies the
mixture-of-experts ridge correction to the *expression* matrix.  This module re-derives
the published algorithm (Korsunsky et al. 2019) with the harmonypy conventions:

* Z_cos = cosine-normalised PCs (after max-scaling), one-hot design Phi (B x N),
  Phi_moe = [1; Phi], lamb = diag([0, lamb...]), K = min(round(N/30), 100) clusters,
  sigma = 0.1, block_size = 0.05, window 3, eps_kmeans 1e-5, eps_harmony 1e-4;
* init: k-means++ (sklearn KMeans(n_init=10, max_iter=25, random_state)) on Z_cos;
* clustering: Y = normalised Z_cos R^T; dist = 2(1 - Y^T Z_cos); R updated block by
  block in a random order (numpy RandomState(random_state), as run_harmony seeds it)
  with the diversity penalty ((E+1)/(O+1))^theta;
* objective = sum R*dist + sigma*sum R log R + cross-entropy term.

On the GPU (harmony.hip) a k-means round is four kinds of launches and no library GEMM:
the centroid product Y = Z_cos R^T as chunked partials with a deterministic reduction,
the blocked R update whose assign kernel forms each cell's distances 2 (1 - Y_k . z_n)
itself (no N x K distance matrix) and accumulates the round's k-means error and entropy,
and one tiny kernel adding the cross-entropy term, which O = R Phi^T reduces to K x B
numbers -- one device-to-host read per round for the convergence test.  Elsewhere
everything except the block order and convergence bookkeeping runs as batched tensor
ops on the GPU.  ``moe_correct_ridge`` is batched over clusters: the K ridge systems
are formed with two GEMMs over cells and the correction is ONE
(features x K(B+1)) x (K(B+1) x cells) GEMM, streamed over cell chunks, instead of the
reference's K sequential rank-(B+1) updates.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from .. import ops


def _design(meta: pd.DataFrame, vars_use) -> tuple[np.ndarray, np.ndarray]:
    if isinstance(vars_use, str):
        vars_use = [vars_use]
    blocks, counts = [], []
    for v in vars_use:
        d = pd.get_dummies(meta[v].astype("category")).to_numpy().T.astype(np.float64)
        blocks.append(d)
        counts.append(d.shape[0])
    return np.vstack(blocks), np.asarray(counts)


class HarmonyResult:
    """harmonypy's result attributes as numpy arrays, copied from the device on first
    access (a 500k-cell R is 400 MB the device pipeline never reads on the host)."""

    _LAZY = ("Z_corr", "Z_cos", "R", "Phi", "Phi_moe", "lamb")

    def __init__(self, tensors: dict | None = None, **kw):
        self._t = dict(tensors or {})
        self.__dict__.update(kw)

    def __getattr__(self, name):
        t = self.__dict__.get("_t", {})
        if name in t:
            v = t[name].cpu().numpy()
            self.__dict__[name] = v
            return v
        raise AttributeError(name)


def _tall_matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A (m, N) @ B (N, n) for a long reduction (N = cells) into a small output (PCs x
    clusters, clusters x batch pairs): one library GEMM gives such a product a single
    output tile -- ONE workgroup walking 500k cells (27 ms per call at N = 500k, m = 50,
    n = 100: profiles/r3aa_harmony_500k_kernel_summary.txt).  Here the reduction is cut
    into ~512 chunks that run as one batched GEMM, then summed in chunk order
    (deterministic)."""
    m, N = A.shape
    n = B.shape[1]
    chunk = max(1024, N // 512)
    nch = N // chunk
    if nch < 4 or A.device.type != "cuda":
        return A @ B
    M = nch * chunk
    A3 = A[:, :M].reshape(m, nch, chunk).transpose(0, 1)
    B3 = B[:M].reshape(nch, chunk, n)
    out = torch.bmm(A3, B3).sum(dim=0)
    if M < N:
        out += A[:, M:] @ B[M:]
    return out


def _entropy_sum(R: torch.Tensor, sigma: torch.Tensor) -> torch.Tensor:
    y = R * torch.log(R)
    y = torch.where(torch.isfinite(y), y, torch.zeros_like(y))
    return (y * sigma[:, None]).sum()


class Harmony:
    def __init__(self, Z, Phi, Phi_moe, Pr_b, sigma, theta, lamb, K, max_iter_harmony=10,
                 max_iter_kmeans=20, epsilon_kmeans=1e-5, epsilon_harmony=1e-4,
                 block_size=0.05, random_state=0, init_backend="sklearn", device=None,
                 verbose=False, phi_n=None):
        dev = torch.device(device) if device is not None else torch.device("cpu")
        dt = torch.float64
        self.dev, self.dt = dev, dt
        self.Z_orig = torch.as_tensor(np.asarray(Z), dtype=dt, device=dev)
        self.Z_corr = self.Z_orig.clone()
        Zc = self.Z_orig / self.Z_orig.max(dim=0).values
        self.Z_cos = Zc / torch.linalg.vector_norm(Zc, dim=0)
        self.Phi = torch.as_tensor(Phi, dtype=dt, device=dev)
        self.Phi_moe = torch.as_tensor(Phi_moe, dtype=dt, device=dev)
        # level structure of the design for the matrix-core ridge kernels (ridge.hip)
        self._lv = _levels(np.asarray(Phi_moe)) if dev.type == "cuda" else None
        self.Pr_b = torch.as_tensor(Pr_b, dtype=dt, device=dev)
        self.sigma = torch.as_tensor(sigma, dtype=dt, device=dev)
        self.theta = torch.as_tensor(theta, dtype=dt, device=dev)
        self.lamb = torch.as_tensor(lamb, dtype=dt, device=dev)
        self.K = int(K)
        self.N = self.Z_orig.shape[1]
        self.window_size = 3
        self.block_size = block_size
        self.max_iter_kmeans = max_iter_kmeans
        self.eps_k, self.eps_h = epsilon_kmeans, epsilon_harmony
        self.rs = np.random.RandomState(random_state)
        self.random_state = random_state
        self.objective_kmeans: list[float] = []
        self.objective_harmony: list[float] = []
        self.kmeans_rounds: list[int] = []
        self.verbose = verbose
        # fused HIP R-update (harmony.hip) needs each cell's batch index per covariate
        self._native = (phi_n is not None and len(phi_n) <= 64 and
                        ops.harmony_native_ok(self.Phi, self.K, self.Phi.shape[0]))
        if self._native:
            offs = np.concatenate([[0], np.cumsum(phi_n)[:-1]]).astype(np.int64)
            Pn = np.asarray(Phi)
            bidx = np.stack([o + Pn[o:o + c].argmax(axis=0) for o, c in zip(offs, phi_n)])
            self.bidx = torch.as_tensor(bidx.astype(np.int32), device=dev).contiguous()
            self._ws: dict = {}
            # fused distances need the centroid table in the assign kernel's LDS and the
            # centroid kernel's d x K outputs (harmony.hip)
            self._fused = ops.harmony_centroids_ok(self.Z_orig.shape[0], self.K)
            self.Zt = self.Z_cos.t().contiguous()              # cells x PCs
            self._obj = torch.zeros(2, dtype=dt, device=dev)    # round's assign sums
            self._obj_out = torch.zeros(1, dtype=dt, device=dev)
        else:
            self._fused = False
        self._init_cluster(init_backend)
        try:
            self._harmonize(max_iter_harmony)
        finally:
            if getattr(self, "_order_next", None) is not None:
                self._order_pool.shutdown(wait=True)
                self._order_next = None

    # ------------------------------------------------------------------ init
    def _init_cluster(self, backend: str):
        from .consensus import kmeans as _km

        X = self.Z_cos.t()
        if self._fused and backend != "sklearn":
            # device k-means init; the centroids by the centroid kernel on a one-hot R
            labels = torch.as_tensor(_km(X, self.K, n_init=10, random_state=self.random_state,
                                         max_iter=25, backend="device",
                                         device_restart_factor=1), device=self.dev)
            onehot = (labels[:, None] == torch.arange(self.K, device=self.dev)[None, :]).to(self.dt)
            Y = ops.harmony_centroids(self.Zt, onehot.contiguous(), self._ws)
            Y = Y / onehot.sum(dim=0).clamp(min=1)[None, :]
            self._init_fused(Y)
            return
        if backend == "sklearn":
            from sklearn.cluster import KMeans

            m = KMeans(n_clusters=self.K, init="k-means++", n_init=10, max_iter=25,
                       random_state=self.random_state)
            m.fit(X.cpu().numpy())
            Y = torch.as_tensor(m.cluster_centers_.T, dtype=self.dt, device=self.dev)
        else:
            # (the consensus step runs 4x the restarts for sklearn-grade optima on a few
            # hundred spectra; here the cells x PCs init only seeds the soft clustering)
            labels = torch.as_tensor(_km(X, self.K, n_init=10, random_state=self.random_state,
                                         max_iter=25, backend="device",
                                         device_restart_factor=1), device=self.dev)
            onehot = (labels[None, :] == torch.arange(self.K, device=self.dev)[:, None]).to(self.dt)
            Y = _tall_matmul(X.t(), onehot.t()) / onehot.sum(dim=1).clamp(min=1)[None, :]
        if self._fused:
            self._init_fused(Y)
            return
        self.Y = Y / torch.linalg.vector_norm(Y, dim=0)
        self._dist()
        R = -self.dist_mat / self.sigma[:, None]
        R = R - R.max(dim=0).values
        R = torch.exp(R)
        self.R = R / R.sum(dim=0)
        if self._native:   # cell-major storage; self.R stays a (K, N) view of it
            self.Rt = self.R.t().contiguous()
            self.R = self.Rt.t()
        self.E = torch.outer(self.R.sum(dim=1), self.Pr_b)
        self.O = _tall_matmul(self.R, self.Phi.t())
        self._objective()
        self.objective_harmony.append(self.objective_kmeans[-1])

    def _init_fused(self, Y: torch.Tensor):
        """Initial soft assignment on the device: one assign pass over every cell with a
        flat penalty (1 / nvar per covariate: R = softmax(-dist / sigma)), which also
        builds E = outer(sum R, Pr_b) and O = R Phi^T from zero and the initial
        objective's terms."""
        self.Y = (Y / torch.linalg.vector_norm(Y, dim=0)).contiguous()
        K, B = self.K, self.Phi.shape[0]
        self.Rt = torch.zeros((self.N, K), dtype=self.dt, device=self.dev)
        self.R = self.Rt.t()
        self.E = torch.zeros((K, B), dtype=self.dt, device=self.dev)
        self.O = torch.zeros((K, B), dtype=self.dt, device=self.dev)
        ws = self._ws
        ws["pen"] = torch.full((K, B), 1.0 / self.bidx.shape[0], dtype=self.dt, device=self.dev)
        cells = torch.arange(self.N, dtype=torch.int32, device=self.dev)
        self._obj.zero_()
        ops.harmony_block_update(self.Rt, None, self.sigma, cells, self.bidx, self.E, self.O,
                                 self.Pr_b, self.theta, ws, Y=self.Y, Zt=self.Zt, obj=self._obj,
                                 steps=(1,))
        self._objective_fused()
        self.objective_harmony.append(self.objective_kmeans[-1])

    def _objective_fused(self):
        ops.harmony_objective(self.O, self.E, self.sigma, self.theta, self._obj, self._obj_out)
        self.objective_kmeans.append(float(self._obj_out.item()))

    def _objective(self):
        if self._fused:
            self._objective_fused()
            return
        kmeans_error = (self.R * self.dist_mat).sum()
        ent = _entropy_sum(self.R, self.sigma)
        x = self.R * self.sigma[:, None]
        z = torch.log((self.O + 1) / (self.E + 1))
        w = (self.theta[None, :] * z) @ self.Phi
        cross = (x * w).sum()
        self.objective_kmeans.append(float(kmeans_error + ent + cross))

    # ------------------------------------------------------------------ loops
    def _harmonize(self, iters: int):
        for _ in range(1, iters + 1):
            self._cluster()
            self.Z_cos, self.Z_corr, self.W = moe_correct_ridge_pcs(
                self.Z_orig, self.R, self.Phi_moe, self.lamb, levels=self._lv)
            if self._fused:
                self.Zt = self.Z_cos.t().contiguous()
            if self._converged(1):
                break

    def _dist(self):
        """dist = 2 (1 - Y^T Z_cos); cell-major (N, K) for the native R update."""
        if self._native:
            self.distT = 2 * (1 - self.Z_cos.t() @ self.Y)
            self.dist_mat = self.distT.t()
        else:
            self.dist_mat = 2 * (1 - self.Y.t() @ self.Z_cos)

    def _cluster(self):
        if not self._fused:
            self._dist()
        i = 0
        for i in range(self.max_iter_kmeans):
            if self._fused:
                Y = ops.harmony_centroids(self.Zt, self.Rt, self._ws)
                self.Y = (Y / torch.linalg.vector_norm(Y, dim=0)).contiguous()
            else:
                Y = _tall_matmul(self.Z_cos, self.R.t())
                self.Y = Y / torch.linalg.vector_norm(Y, dim=0)
                self._dist()
            self._update_R()
            self._objective()
            if i > self.window_size and self._converged(0):
                break
        self.kmeans_rounds.append(i)
        self.objective_harmony.append(self.objective_kmeans[-1])

    def _shuffled(self):
        """The next round's block order (RandomState.shuffle of 0..N-1, the k-th call
        for the k-th round whichever thread runs it) as pinned int32."""
        order = np.arange(self.N)
        self.rs.shuffle(order)
        t = torch.from_numpy(order.astype(np.int32))
        return t.pin_memory() if self.dev.type == "cuda" else t

    def _update_R(self):
        order = np.arange(self.N)
        if self._native:
            # the shuffle of 500k indices is ~10 ms of host time per round: the next
            # round's order is drawn on a helper thread while the GPU runs this one (same
            # RandomState sequence -- the draws stay in round order)
            if getattr(self, "_order_next", None) is None:
                import concurrent.futures as cf

                self._order_pool = cf.ThreadPoolExecutor(max_workers=1)
                self._order_next = self._order_pool.submit(self._shuffled)
            order_h = self._order_next.result()
            self._order_next = self._order_pool.submit(self._shuffled)
            n_blocks = int(math.ceil(1 / self.block_size))
            self.E = self.E.contiguous()
            self.O = self.O.contiguous()
            # one host->device copy of the round's order; blocks are device slices of it
            order_d = order_h.to(self.dev, non_blocking=True)
            a = 0
            for size in (len(b) for b in np.array_split(np.empty(self.N, np.int8), n_blocks)):
                cells = order_d[a:a + size]
                a += size
                if self._fused:
                    ops.harmony_block_update(self.Rt, None, self.sigma, cells, self.bidx,
                                             self.E, self.O, self.Pr_b, self.theta, self._ws,
                                             Y=self.Y, Zt=self.Zt, obj=self._obj)
                else:
                    ops.harmony_block_update(self.Rt, self.distT, self.sigma, cells, self.bidx,
                                             self.E, self.O, self.Pr_b, self.theta, self._ws)
            return
        sd = -self.dist_mat / self.sigma[:, None]
        sd = sd - sd.max(dim=0).values
        sd = torch.exp(sd)
        self.rs.shuffle(order)
        n_blocks = int(math.ceil(1 / self.block_size))
        for b in np.array_split(order, n_blocks):
            bi = torch.as_tensor(b, device=self.dev)
            Rb = self.R[:, bi]
            Pb = self.Phi[:, bi]
            self.E -= torch.outer(Rb.sum(dim=1), self.Pr_b)
            self.O -= Rb @ Pb.t()
            pen = torch.pow((self.E + 1) / (self.O + 1), self.theta[None, :]) @ Pb
            Rn = sd[:, bi] * pen
            Rn = Rn / Rn.abs().sum(dim=0)
            self.R[:, bi] = Rn
            self.E += torch.outer(Rn.sum(dim=1), self.Pr_b)
            self.O += Rn @ Pb.t()

    def _converged(self, kind: int) -> bool:
        if kind == 0:
            ok = self.objective_kmeans
            n = len(ok)
            old = sum(ok[n - 2 - i] for i in range(self.window_size))
            new = sum(ok[n - 1 - i] for i in range(self.window_size))
            return abs(old - new) / abs(old) < self.eps_k
        old, new = self.objective_harmony[-2], self.objective_harmony[-1]
        return (old - new) / abs(old) < self.eps_h

    def result(self) -> HarmonyResult:
        return HarmonyResult(dict(Z_corr=self.Z_corr, Z_cos=self.Z_cos, R=self.R, Phi=self.Phi,
                                  Phi_moe=self.Phi_moe, lamb=self.lamb), K=self.K,
                             objective_harmony=list(self.objective_harmony),
                             kmeans_rounds=list(self.kmeans_rounds), _R_t=self.R,
                             _Phi_moe_t=self.Phi_moe, _lamb_t=self.lamb, _lv=self._lv)


def run_harmony(data_mat, meta_data: pd.DataFrame, vars_use, theta=None, lamb=None,
                sigma=0.1, nclust=None, tau=0, block_size=0.05, max_iter_harmony=10,
                max_iter_kmeans=20, epsilon_cluster=1e-5, epsilon_harmony=1e-4,
                random_state=0, init_backend="sklearn", device=None, verbose=False):
    """harmonypy.run_harmony equivalent (cells x dims or dims x cells input)."""
    N = meta_data.shape[0]
    Z = np.asarray(data_mat, dtype=np.float64)
    if Z.shape[1] != N:
        Z = Z.T
    if Z.shape[1] != N:
        raise ValueError("data_mat and meta_data do not have the same number of cells")
    if nclust is None:
        nclust = int(min(round(N / 30.0), 100))
    sigma = np.repeat(float(sigma), nclust) if np.isscalar(sigma) else np.asarray(sigma)
    Phi, phi_n = _design(meta_data, vars_use)
    if theta is None:
        theta = np.repeat([1.0] * len(phi_n), phi_n)
    elif np.isscalar(theta):
        theta = np.repeat([float(theta)] * len(phi_n), phi_n)
    else:
        theta = np.repeat(np.asarray(theta, dtype=float), phi_n)
    if lamb is None:
        lamb = np.repeat([1.0] * len(phi_n), phi_n)
    elif np.isscalar(lamb):
        lamb = np.repeat([float(lamb)] * len(phi_n), phi_n)
    else:
        lamb = np.repeat(np.asarray(lamb, dtype=float), phi_n)
    N_b = Phi.sum(axis=1)
    Pr_b = N_b / N
    if tau > 0:
        theta = theta * (1 - np.exp(-(N_b / (nclust * tau)) ** 2))
    lamb_mat = np.diag(np.insert(lamb, 0, 0))
    Phi_moe = np.vstack((np.ones((1, N)), Phi))
    ho = Harmony(Z, Phi, Phi_moe, Pr_b, sigma, theta, lamb_mat, nclust, max_iter_harmony,
                 max_iter_kmeans, epsilon_cluster, epsilon_harmony, block_size, random_state,
                 init_backend, device, verbose, phi_n=phi_n)
    return ho.result()


def _ridge_weights(Z: torch.Tensor, R: torch.Tensor, Phi_moe: torch.Tensor, lamb: torch.Tensor,
                   chunk: int = 65536) -> torch.Tensor:
    """W_k = (Phi_Rk Phi_moe^T + lamb)^-1 Phi_Rk Z^T for all clusters; W_k[0] = 0.
    Returns (K*(B+1), F) with Z (F x N)."""
    K, N = R.shape
    B1 = Phi_moe.shape[0]
    F = Z.shape[0]
    # sum_n R[k,n] P[b,n] P[c,n] via pair products: (K x N) @ (N x B1*B1)
    PP = (Phi_moe[:, None, :] * Phi_moe[None, :, :]).reshape(B1 * B1, N)
    A = _tall_matmul(R, PP.t()).reshape(K, B1, B1) + lamb[None]
    Y = torch.zeros((K * B1, F), dtype=Z.dtype, device=Z.device)
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        RP = (R[:, None, a:b] * Phi_moe[None, :, a:b]).reshape(K * B1, b - a)
        Y += _tall_matmul(RP, Z[:, a:b].t())
    W = torch.linalg.solve(A, Y.view(K, B1, F))
    W[:, 0, :] = 0
    return W.reshape(K * B1, F)


def _apply_correction(Z: torch.Tensor, W: torch.Tensor, R: torch.Tensor, Phi_moe: torch.Tensor,
                      chunk: int = 65536) -> torch.Tensor:
    K, N = R.shape
    B1 = Phi_moe.shape[0]
    out = Z.clone()
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        RP = (R[:, None, a:b] * Phi_moe[None, :, a:b]).reshape(K * B1, b - a)
        out[:, a:b] -= W.t() @ RP
    return out


def moe_correct_ridge_pcs(Z_orig: torch.Tensor, R: torch.Tensor, Phi_moe: torch.Tensor,
                          lamb: torch.Tensor, levels=None):
    if levels is not None and Z_orig.is_cuda and ops.use_native(Z_orig):
        # the PCs (d x N) through the level-segment kernels (ridge.hip), cells x d
        Zc, Wk = _ridge_native(Z_orig.t().contiguous(), R.t().contiguous(), levels, lamb,
                               return_w=True)
        Z_corr = Zc.t()
        Z_cos = Z_corr / torch.linalg.vector_norm(Z_corr, dim=0)
        return Z_cos, Z_corr, Wk.reshape(-1, Wk.shape[2])
    W = _ridge_weights(Z_orig, R, Phi_moe, lamb)
    Z_corr = _apply_correction(Z_orig, W, R, Phi_moe)
    Z_cos = Z_corr / torch.linalg.vector_norm(Z_corr, dim=0)
    return Z_cos, Z_corr, W


def moe_correct_ridge(Z_orig, Z_cos, Z_corr, R, W, K, Phi_Rk, Phi_moe, lamb, device=None,
                      dtype=torch.float64):
    """preprocess.py:9-18 signature: returns (Z_cos, Z_corr, W_last, Phi_Rk_last) for a
    features x cells matrix ``Z_orig`` (numpy in, numpy out)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    Zt = torch.as_tensor(np.asarray(Z_orig), dtype=dtype, device=dev)
    Rt = torch.as_tensor(np.asarray(R), dtype=dtype, device=dev)[:int(K)]
    Pt = torch.as_tensor(np.asarray(Phi_moe), dtype=dtype, device=dev)
    Lt = torch.as_tensor(np.asarray(lamb), dtype=dtype, device=dev)
    Wall = _ridge_weights(Zt, Rt, Pt, Lt)
    Zc = _apply_correction(Zt, Wall, Rt, Pt)
    Zcos = Zc / torch.linalg.vector_norm(Zc, dim=0)
    B1 = Pt.shape[0]
    W_last = Wall[(int(K) - 1) * B1:].cpu().numpy()
    Phi_Rk = (Pt * Rt[int(K) - 1]).cpu().numpy()
    return Zcos.cpu().numpy(), Zc.cpu().numpy(), W_last, Phi_Rk


def _host(a) -> np.ndarray:
    return a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


def _levels(Phi_moe: np.ndarray):
    """Level structure of a Harmony design [1; one-hot levels] (B1 x N): per row b the
    cells of that level, and per cell its combination of levels (plus a per-device cache
    of the index tensors the kernels read).  None when Phi_moe is not of that form (the
    dense path then applies)."""
    P = np.asarray(Phi_moe)
    if P.ndim != 2 or P.shape[0] < 1 or not np.all(P[0] == 1.0) or \
            not np.all((P == 0.0) | (P == 1.0)):
        return None
    B1, N = P.shape
    cells = [np.arange(N)] + [np.flatnonzero(P[b]) for b in range(1, B1)]
    # a cell's combination of levels as one integer: its level rows (ascending) in base B1
    # -- a 1-D unique (np.unique(axis=0) over the N x B one-hot rows lexsorts them: ~1 s of
    # the 500k-cell Harmony stage, profiles/r4d_*)
    lab = np.zeros(N, dtype=np.int64)
    cnt = np.zeros(N, dtype=np.int64)
    for b in range(1, B1):
        on = cells[b]
        lab[on] = lab[on] * B1 + b
        cnt[on] += 1
    m = int(cnt.max()) if N else 0
    if N and (cnt.min() != m or m * np.log2(max(B1, 2)) > 62):
        keys, inv = np.unique(P[1:].T.astype(np.uint8), axis=0, return_inverse=True)
        lev = [np.flatnonzero(row) + 1 for row in keys]
    else:
        ukeys, inv = np.unique(lab, return_inverse=True)
        lev = []
        for v in ukeys.tolist():
            rows = []
            for _ in range(m):
                rows.append(v % B1)
                v //= B1
            lev.append(np.asarray(rows[::-1], dtype=np.int64))
    inv = np.asarray(inv).reshape(-1)
    if len(lev) > 4096:
        return None
    return {"cells": cells, "inv": inv, "lev": lev, "N": N, "B1": B1, "dev": {}}


def _level_tensors(lv: dict, dev: torch.device) -> dict:
    """Device index tensors of a level structure (built once per device)."""
    key = str(dev)
    t = lv["dev"].get(key)
    if t is not None:
        return t
    cells, inv, lev = lv["cells"], lv["inv"], lv["lev"]
    B1, N = lv["B1"], lv["N"]
    Pm = np.zeros((N, B1))
    for b, cl in enumerate(cells):
        Pm[cl, b] = 1.0
    L = max(len(v) for v in lev)
    tab = np.zeros((len(lev), L), dtype=np.int64)
    for c, v in enumerate(lev):
        tab[c, :len(v)] = v
    order = np.argsort(inv, kind="stable").astype(np.int32)
    cnt = np.bincount(inv, minlength=len(lev))
    starts = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    blk = [(c, int(starts[c]) + o, int(min(64, cnt[c] - o)))
           for c in range(len(lev)) for o in range(0, int(cnt[c]), 64)]
    t = {"idx": torch.from_numpy(np.concatenate(cells).astype(np.int32)).to(dev),
         "seg": torch.from_numpy(np.concatenate([[0], np.cumsum([c.size for c in cells])])
                                 .astype(np.int64)).to(dev),
         "Pt": torch.from_numpy(Pm).to(dev),
         "tab": torch.from_numpy(tab).to(dev),
         "order": torch.from_numpy(order).to(dev),
         "blk": torch.from_numpy(np.asarray(blk, dtype=np.int32).reshape(-1)).to(dev),
         "nblk": len(blk)}
    lv["dev"][key] = t
    return t


# workgroups a ridge_seg_tgemm launch should have before the levels are cut into chunks
# (256 CUs; the kernel is one 4-wave workgroup per (segment, 32 clusters, 64 features))
_SEG_TARGET_WG = 2048


def _seg_chunks(lv: dict, t: dict, tiles: int, dev: torch.device):
    """Chunk table for a ridge_seg_tgemm with ``tiles`` (cluster x feature) tiles per
    segment: (chunk boundaries into the level cell list (int64, nchunk + 1), first chunk
    of every level (int32, B1 + 1), nchunk), or None when the levels alone fill the chip."""
    B1 = lv["B1"]
    if B1 * tiles >= _SEG_TARGET_WG:
        return None
    seg = np.concatenate([[0], np.cumsum([c.size for c in lv["cells"]])]).astype(np.int64)
    want = -(-_SEG_TARGET_WG // tiles)
    size = max(256, -(-int(seg[-1]) // want))
    size = -(-size // 16) * 16               # whole 4-cell steps of the 4 waves
    key = ("chunks", size)
    c = t.get(key)
    if c is None:
        bounds, first = [], [0]
        for b in range(B1):
            s0, s1 = int(seg[b]), int(seg[b + 1])
            starts = list(range(s0, s1, size)) or [s0]
            bounds.extend(starts)
            first.append(first[-1] + len(starts))
        bounds.append(int(seg[-1]))
        c = (torch.from_numpy(np.asarray(bounds, dtype=np.int64)).to(dev),
             torch.from_numpy(np.asarray(first, dtype=np.int32)).to(dev), len(bounds) - 1)
        t[key] = c
    return c


def _seg_tgemm(h, lv, t, Rt, Kc, X, ldx, F, x_f64, out, st):
    """out[b][k][f] = sum over level b's cells of R[k, n] X[n, f] (out: B1 x Kc x F)."""
    B1 = lv["B1"]
    tiles = -(-Kc // 32) * -(-F // 64)
    ch = _seg_chunks(lv, t, tiles, X.device if isinstance(X, torch.Tensor) else Rt.device)
    xp = X.data_ptr()
    if ch is None:
        h.ridge_seg_tgemm(Rt.data_ptr(), Rt.stride(0), Kc, xp, x_f64, ldx, F,
                          t["idx"].data_ptr(), t["seg"].data_ptr(), B1, out.data_ptr(),
                          Kc * F, F, st)
        return
    bounds, first, nch = ch
    part = torch.empty((nch, Kc, F), dtype=torch.float64, device=out.device)
    h.ridge_seg_tgemm(Rt.data_ptr(), Rt.stride(0), Kc, xp, x_f64, ldx, F, t["idx"].data_ptr(),
                      bounds.data_ptr(), nch, part.data_ptr(), Kc * F, F, st)
    h.ridge_seg_reduce(part.data_ptr(), first.data_ptr(), B1, Kc, F, out.data_ptr(), Kc * F, F,
                       st)


def _ridge_native(X: torch.Tensor, Rt: torch.Tensor, lv: dict, Lt: torch.Tensor,
                  return_w: bool = False):
    """The MOE ridge correction on the f64 matrix cores (csrc/kernels/ridge.hip) for a
    cells x features X and R^T (cells x clusters): level-segment products for Y and the
    ridge Grams, float64 solves of the (B+1) x (B+1) systems on the host (no library
    GEMM), one combination-grouped correction pass rounded once."""
    h = ops._hip
    dev = X.device
    t = _level_tensors(lv, dev)
    N, F = X.shape
    Kc = Rt.shape[1]
    B1 = lv["B1"]
    st = ops._stream_ptr(X)
    # Y[b][k][f] = sum over level b's cells of R[k, n] X[n, f]
    Y = torch.empty((B1, Kc, F), dtype=torch.float64, device=dev)
    _seg_tgemm(h, lv, t, Rt, Kc, X, X.stride(0), F, int(X.dtype == torch.float64), Y, st)
    # A0[b][k][c] = sum over level b's cells of R[k, n] Phi[c, n]
    Pt = t["Pt"]
    A0 = torch.empty((B1, Kc, B1), dtype=torch.float64, device=dev)
    _seg_tgemm(h, lv, t, Rt, Kc, Pt, Pt.stride(0), B1, 1, A0, st)
    A = A0.permute(1, 0, 2).cpu().numpy() + Lt.cpu().numpy()[None]        # (Kc, B1, B1)
    Wh = np.linalg.solve(A, Y.permute(1, 0, 2).cpu().numpy())               # (Kc, B1, F)
    Wh[:, 0, :] = 0.0                                    # keep the intercept
    W = torch.from_numpy(Wh).to(dev)
    # per level combination: Wc = sum of its levels' W_b (W_0 = 0 pads short lists)
    tab = t["tab"]
    Wc = torch.zeros((tab.shape[0], Kc, F), dtype=torch.float64, device=dev)
    Wp = W.permute(1, 0, 2)                              # (B1, Kc, F) view
    for j in range(tab.shape[1]):
        Wc += Wp.index_select(0, tab[:, j])
    out = torch.empty_like(X)
    h.ridge_apply(Rt.data_ptr(), Rt.stride(0), Kc, X.data_ptr(), int(X.dtype == torch.float64),
                  X.stride(0), out.data_ptr(), out.stride(0), F, t["order"].data_ptr(),
                  t["blk"].data_ptr(), t["nblk"], Wc.data_ptr(), Kc * F, F, st)
    return (out, W) if return_w else out


def moe_correct_expression(X: torch.Tensor, R, Phi_moe, lamb, K: int | None = None,
                           chunk: int = 65536, levels=None) -> torch.Tensor:
    """The MOE ridge correction of preprocess.py:9-18 applied to a device-resident
    (cells x features) expression matrix, in place of the features x cells numpy
    round trip: W_k = (Phi_Rk Phi_moe^T + lamb)^-1 Phi_Rk X (W_k[0] = 0, intercept kept),
    X -= sum_k Phi_Rk^T W_k -- batched over clusters into GEMMs streamed over cell
    chunks, float64 arithmetic, result stored in X's dtype (numpy's in-place
    float32 -= float64 of the reference).  Returns the corrected matrix (new tensor)."""
    dev = X.device
    # (device tensors -- Harmony's own R / lamb -- are taken as they are, no host trip)
    Rt = torch.as_tensor(R, dtype=torch.float64, device=dev)
    if K is not None:
        Rt = Rt[:int(K)]
    Lt = torch.as_tensor(lamb, dtype=torch.float64, device=dev)
    if dev.type == "cuda" and ops.use_native(X) and X.dtype in (torch.float32, torch.float64) \
            and X.dim() == 2 and (X.shape[1] <= 1 or X.stride(1) == 1):
        lv = levels if levels is not None else _levels(_host(Phi_moe))
        if lv is not None:   # the f64 matrix-core kernels (no materialised Phi_Rk)
            return _ridge_native(X, Rt.t().contiguous(), lv, Lt)
    Pt = torch.as_tensor(Phi_moe, dtype=torch.float64, device=dev)
    Kc, N = Rt.shape
    B1 = Pt.shape[0]
    F = X.shape[1]
    PP = (Pt[:, None, :] * Pt[None, :, :]).reshape(B1 * B1, N)
    A = (Rt @ PP.t()).reshape(Kc, B1, B1) + Lt[None]
    Y = torch.zeros((Kc * B1, F), dtype=torch.float64, device=dev)
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        RP = (Rt[:, None, a:b] * Pt[None, :, a:b]).reshape(Kc * B1, b - a)
        Y += RP @ X[a:b].to(torch.float64)
    W = torch.linalg.solve(A, Y.view(Kc, B1, F))
    W[:, 0, :] = 0
    W = W.reshape(Kc * B1, F)
    out = torch.empty_like(X)
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        RP = (Rt[:, None, a:b] * Pt[None, :, a:b]).reshape(Kc * B1, b - a)
        out[a:b] = (X[a:b].to(torch.float64) - RP.t() @ W).to(X.dtype)
    return out

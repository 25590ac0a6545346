"""Consensus-step algorithms (C24, cnmf.py:1053-1110).

All run on the device of their input tensor (HIP GPU or CPU):

* ``l2_normalize_rows``       -- H1, rows scaled to unit L2 norm (cnmf.py:1056)
* ``pairwise_distances``      -- H2, ||a||^2 + ||b||^2 - 2 a.b^T on the matrix cores
* ``local_density``           -- H3, mean distance to the n_neighbors nearest (self
                                 included in the n+1 smallest, divided by n; cnmf.py:1067-1070)
* ``kmeans``                  -- H4, k-means++ init + Lloyd, ``n_init`` restarts batched,
                                 best inertia (sklearn semantics).  ``backend='sklearn'``
                                 reproduces ``KMeans(n_clusters=k, n_init=10, random_state=1)``
                                 of cnmf.py:1082 exactly (CPU); ``'device'`` runs on the GPU.
* ``cluster_medians``         -- H5, per-cluster per-gene median, rows renormalised to 1
* ``silhouette``              -- H6, from the same distance matrix (segmented row sums)
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import ops


def l2_normalize_rows(S: torch.Tensor) -> torch.Tensor:
    return S / torch.sqrt((S * S).sum(dim=1, keepdim=True))


def pairwise_distances(A: torch.Tensor, B: torch.Tensor | None = None) -> torch.Tensor:
    """Euclidean distances in float64 (sklearn semantics: clipped at 0, exact zeros on the
    diagonal when B is A).  GPU: f64 MFMA kernel (ops.pairwise_dist)."""
    return ops.pairwise_dist(A, B)


def local_density(dist: torch.Tensor, n_neighbors: int) -> torch.Tensor:
    """Mean distance to the ``n_neighbors`` nearest neighbours (cnmf.py:1065-1070):
    sum of the (n_neighbors+1) smallest distances of each row (self included) / n_neighbors.
    GPU: exact radix-select kernel (ops.knn_sum)."""
    k = min(n_neighbors + 1, dist.shape[1])
    tot = ops.knn_sum(dist, k)
    return tot / max(n_neighbors, 1) if n_neighbors > 0 else tot * float("inf")


# ------------------------------------------------------------------------- k-means
def _kmeanspp(X: torch.Tensor, k: int, gen: torch.Generator, x_sq: torch.Tensor) -> torch.Tensor:
    """Greedy k-means++ (sklearn _kmeans_plusplus, n_local_trials = 2 + log k), one
    restart (the CPU path; the GPU runs every restart at once in _kmeanspp_batched)."""
    return _kmeanspp_batched(X, k, gen, 1)[0]


def _kmeanspp_batched(X: torch.Tensor, k: int, gen: torch.Generator, n_init: int) -> torch.Tensor:
    """Greedy k-means++ for ``n_init`` restarts at once (sklearn _kmeans_plusplus with
    n_local_trials = 2 + log k): every centre step scores all restarts' candidates with
    ONE distance launch (n x n_init*trials, f64 MFMA), and the candidate sampling (inverse
    CDF of each restart's potential) stays on the device -- the uniforms are drawn up
    front from the host generator, so there is no device->host sync per centre.
    Returns (n_init, k, d)."""
    n, d = X.shape
    dev = X.device
    trials = 2 + int(math.log(k))
    first = torch.randint(n, (n_init,), generator=gen)
    u = torch.rand((max(k - 1, 0), n_init, trials), generator=gen, dtype=torch.float64)
    first, u = first.to(dev), u.to(dev)
    centers = torch.empty((n_init, k, d), dtype=X.dtype, device=dev)
    centers[:, 0] = X[first]
    closest = ops.pairwise_dist(X, X[first], squared=True)           # (n, n_init)
    ar = torch.arange(n_init, device=dev)
    # Large n in few dimensions (Harmony's init: 500k cells x 20 PCs, 100 centres x 10
    # restarts x 6 trials): the fused kernel scores every candidate without the
    # (n x n_init*trials) float64 distance matrix, which cost ~1 GB of HBM traffic per
    # centre (kmeans.hip kmeanspp_kernel).  Few points (consensus spectra): one MFMA
    # distance launch per centre.
    fused = n > 4096 and ops.kmeanspp_fused_ok(X, n_init * trials)
    if fused:
        closest = closest.contiguous()
    for c in range(1, k):
        if fused:
            # inverse CDF of each restart's potential (block sums + one workgroup per
            # restart, kmeans.hip ppsample_kernel)
            cand = ops.kmeanspp_sample(closest, u[c - 1])
        else:
            # the scan runs along the contiguous dimension ((n_init, n) layout: the
            # outer-dimension scan of an (n, n_init) tensor took 40 ms per centre at 200k)
            cum = torch.cumsum(closest.t().contiguous().double(), 1)  # (n_init, n)
            r = u[c - 1] * cum[:, -1:]                                # (n_init, trials)
            cand = torch.searchsorted(cum, r).clamp(max=n - 1)
        if fused:
            pot = ops.kmeanspp_step(X, X[cand.reshape(-1)], closest, trials)
            best = torch.argmin(pot, dim=1)                           # (n_init,)
            ops.kmeanspp_step(X, X[cand[ar, best]], closest, 1, update=True)
        else:
            dcand = ops.pairwise_dist(X, X[cand.reshape(-1)], squared=True)
            dcand = dcand.view(n, n_init, trials)
            newc = torch.minimum(closest[:, :, None], dcand)          # (n, n_init, trials)
            best = torch.argmin(newc.sum(dim=0), dim=1)               # (n_init,)
            closest = newc[:, ar, best]
        centers[:, c] = X[cand[ar, best]]
    return centers


def _lloyd_batched(X: torch.Tensor, centers: torch.Tensor, max_iter: int, tol: float):
    """Lloyd iterations for all restarts at once: centers (n_init, k, d).  Assignment is
    one f64 MFMA distance launch over the n_init*k centroids + a segmented argmin
    (ops.seg_argmin); restarts that stop moving (shift <= tol) are frozen.
    Returns (labels (n, n_init), inertia (n_init,))."""
    n_init, k, d = centers.shape
    n = X.shape[0]
    if ops.kmeans_fused_ok(X, k):
        return _lloyd_fused(X, centers, max_iter, tol)
    live = torch.ones(n_init, dtype=torch.bool, device=X.device)
    ones = torch.ones((n_init, n), dtype=torch.float64, device=X.device)
    for it in range(max_iter):
        C = centers.reshape(n_init * k, d)
        lab, _ = ops.seg_argmin(ops.pairwise_dist(X, C, squared=True), k)
        # cluster sums of every restart in one segmented-sum launch (segsum.hip: float64,
        # points summed in index order -- no one-hot matrix, no library GEMM)
        labT = lab.t().contiguous()                                   # (n_init, n)
        sums = ops.seg_colsum(X, labT, k)                              # (n_init, k, d)
        counts = torch.zeros((n_init, k), dtype=torch.float64, device=X.device)
        counts.scatter_add_(1, labT, ones)                             # exact (integers)
        newc = torch.where(counts[..., None] > 0,
                           sums / counts.clamp(min=1)[..., None], centers).to(X.dtype)
        shift = ((newc - centers) ** 2).sum(dim=(1, 2))
        centers = torch.where(live[:, None, None], newc, centers)
        live = live & (shift > tol)
        # frozen restarts keep their centres, so checking every 4th step only costs a
        # few no-op steps; it spares 3 of 4 host syncs
        if it % 4 == 3 and not bool(live.any()):
            break
    lab, mind = ops.seg_argmin(ops.pairwise_dist(X, centers.reshape(n_init * k, d),
                                                 squared=True), k)
    return lab, mind.sum(dim=0)


def _lloyd_fused(X: torch.Tensor, centers: torch.Tensor, max_iter: int, tol: float):
    """Low-dimensional Lloyd (d <= 64, e.g. Harmony's k-means init on cells x PCs): one
    fused assign+accumulate launch per iteration for every restart (ops.kmeans_step,
    kmeans.hip) -- no (n x n_init*k) distance matrix, no atomics; same freezing rule."""
    n_init, k, d = centers.shape
    live = torch.ones(n_init, dtype=torch.bool, device=X.device)
    for _ in range(max_iter):
        _, sums, counts, _ = ops.kmeans_step(X, centers, live=live)
        newc = torch.where(counts[..., None] > 0, sums / counts.clamp(min=1)[..., None], centers)
        shift = ((newc - centers) ** 2).sum(dim=(1, 2))
        centers = torch.where(live[:, None, None], newc, centers)
        live = live & (shift > tol)
        if not bool(live.any()):
            break
    lab, _, _, mind = ops.kmeans_step(X, centers, want_sums=False, want_dist=True)
    return lab.t(), mind.sum(dim=1)


def kmeans(X, k: int, n_init: int = 10, random_state: int = 1, max_iter: int = 300,
           tol: float = 1e-4, backend: str = "auto", device_restart_factor: int = 4):
    """Returns integer labels 0..k-1 (numpy).  ``backend='sklearn'`` is the reference's
    KMeans(n_clusters=k, n_init=10, random_state=1) (cnmf.py:1082) bit for bit;
    ``'device'`` runs batched k-means++ + batched Lloyd (same algorithm, own RNG stream)
    on the tensor's device (HIP kernels); ``'auto'`` (default) = device for GPU tensors,
    sklearn otherwise.  The device path runs ``device_restart_factor`` x ``n_init``
    restarts: they share the same launches (nearly free), and with its own RNG stream 10
    restarts reached sklearn's best inertia less often (5/10 vs 9/10 seeds on the K=8
    golden spectra of tests/data; 40 restarts: 10/10)."""
    if backend == "auto":
        backend = "device" if isinstance(X, torch.Tensor) and X.device.type == "cuda" \
            else "sklearn"
    if backend == "sklearn":
        from sklearn.cluster import KMeans

        Xn = X.detach().cpu().numpy() if isinstance(X, torch.Tensor) else np.asarray(X)
        m = KMeans(n_clusters=k, n_init=n_init, random_state=random_state)
        m.fit(Xn)
        return m.labels_
    Xt = X if isinstance(X, torch.Tensor) else torch.as_tensor(np.asarray(X))
    Xt = Xt.to(torch.float64)
    # sklearn scales tol by the mean feature variance
    tol_abs = tol * float(Xt.var(dim=0, unbiased=False).mean())
    gen = torch.Generator(device="cpu").manual_seed(int(random_state))
    c0 = _kmeanspp_batched(Xt, k, gen, n_init * max(1, int(device_restart_factor)))
    labels, inertia = _lloyd_batched(Xt, c0, max_iter, tol_abs)
    best = int(torch.argmin(inertia))
    return labels[:, best].cpu().numpy()


def cluster_medians(S: torch.Tensor, labels: np.ndarray, k_labels) -> torch.Tensor:
    """Per-cluster per-gene median (pandas groupby().median() semantics: mean of the two
    middle values for even counts), rows renormalised to sum 1 (cnmf.py:1087-1090).

    Segmented on the device with no loop over clusters: every gene column is sorted by
    value, then stably by cluster, so each cluster's values form an ascending segment and
    its median sits at fixed offsets of the segment -- two sorts and gathers for all
    clusters and genes at once, exact."""
    lab = np.asarray(labels)
    order = {c: i for i, c in enumerate(k_labels)}
    rank = np.array([order.get(c, -1) for c in lab], dtype=np.int64)
    keep = rank >= 0
    R = S if keep.all() else S[torch.as_tensor(np.flatnonzero(keep), device=S.device)]
    rk = rank[keep]
    counts = np.bincount(rk, minlength=len(k_labels))
    if (counts == 0).any():
        raise ValueError("cluster_medians: an empty cluster")
    if R.dtype == torch.float64:
        # GPU: one workgroup per gene ranks every value inside its cluster in LDS
        # (seg_median.hip) -- no sort; beyond its limits the sorts below
        med = ops.seg_median(R if R.stride(-1) == 1 else R.contiguous(), rk, len(k_labels))
        if med is not None:
            return med / med.sum(dim=1, keepdim=True)
    vals, i1 = torch.sort(R, dim=0)                                   # by value, per gene
    lab_t = torch.as_tensor(rk, device=S.device)
    _, i2 = torch.sort(lab_t[i1], dim=0, stable=True)                 # then by cluster
    seg = torch.gather(vals, 0, i2)
    start = np.concatenate([[0], np.cumsum(counts)[:-1]])
    lo_i = torch.as_tensor(start + (counts - 1) // 2, device=S.device)
    hi_i = torch.as_tensor(start + counts // 2, device=S.device)
    med = 0.5 * (seg[lo_i] + seg[hi_i])
    return med / med.sum(dim=1, keepdim=True)


def silhouette(dist: torch.Tensor, labels: np.ndarray) -> float:
    """Mean silhouette coefficient from a precomputed distance matrix (sklearn semantics:
    singleton clusters score 0)."""
    lab = torch.as_tensor(np.asarray(labels), device=dist.device)
    uniq, own = torch.unique(lab, return_inverse=True)
    # per-row cluster sums of the distances (segsum.hip: float64, fixed order, no GEMM)
    sums = ops.seg_rowsum(dist, own, len(uniq))                    # n x c
    counts = torch.bincount(own, minlength=len(uniq)).to(torch.float64)
    own_cnt = counts[own]
    a = sums[torch.arange(len(lab)), own] / torch.clamp(own_cnt - 1, min=1)
    other = sums / counts[None, :]
    other[torch.arange(len(lab)), own] = float("inf")
    b = other.min(dim=1).values
    s = (b - a) / torch.maximum(a, b)
    s = torch.where(own_cnt > 1, s, torch.zeros_like(s))
    s = torch.nan_to_num(s, nan=0.0)
    return float(s.mean())

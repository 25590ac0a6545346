"""Background first-use loading of the device code the later pipeline stages call.

HIP loads a kernel's code object on its first launch in a process.  For the small
consensus / k-selection kernels that load, not the work, is the cost: one K's
k-selection statistics take 26 ms warm and 1.0 s on the first call of a process
(``profiles/r5ze_kstats_{warm,cold}.txt``: the first ``pow`` / ``minimum`` / ``clamp`` /
``sqrt`` / ``unique`` each ~0.05-0.13 s, the first f32 / f64 library GEMM another ~0.15 s).
``start`` runs those stages' building blocks once on tiny inputs, on a thread of its own
and a stream of its own, while the caller's stage (``cNMF.prepare``) does its own work;
``wait`` joins it.  Best effort: a failure here only leaves a first call cold.

Nothing cooperative runs here (no solve: a cooperative launch must not share the GPU with
another one), and the caller joins before any later stage could capture a HIP graph.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from .log import get_logger

log = get_logger("cnmf_torch_amd.prewarm")

_LOCK = threading.Lock()
_THREADS: dict = {}
errors: list = []       # (what, repr of the exception) of background work that stopped


def start(device, parallel: bool = False) -> list:
    """Start warming ``device`` (once per process and device): the groups below all on
    one thread (default), or on one thread each (``parallel``: the code-object loads
    overlap, 0.24 s against 0.53 s, but the shorter prepare then leaves the figure
    process's matplotlib import running under factorize, whose host-bound stage time
    varied 0.094-0.125 s against 0.095-0.100 s: profiles/r5zj_*, r5zk_*).  [] off the
    GPU."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return []
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _LOCK:
        ts = _THREADS.get(idx)
        if ts is None:
            d = torch.device("cuda", idx)
            groups = [[g] for g in _GROUPS] if parallel else [list(_GROUPS)]
            ts = [threading.Thread(target=_run, args=(d, grp), name="cnmf-prewarm",
                                   daemon=True) for grp in groups]
            _THREADS[idx] = ts
            for t in ts:
                t.start()
    return ts


_EXTRA: list = []


def run(device, fn) -> threading.Thread | None:
    """Run ``fn()`` now on a background thread with a stream of its own (device work a
    later stage of this process will reuse, e.g. the data matrix's GEMM planes);
    joined -- and its stream drained -- by :func:`wait`.  None off the GPU."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return None

    def body():
        try:
            with torch.cuda.device(dev):
                s = torch.cuda.Stream(dev)
                with torch.cuda.stream(s):
                    fn()
                s.synchronize()
        except Exception as e:      # best effort: the later stage builds it itself
            errors.append(("build", repr(e)))
            log.debug("background build stopped: %s", e)

    t = threading.Thread(target=body, name="cnmf-prebuild", daemon=True)
    with _LOCK:
        _EXTRA.append(t)
    t.start()
    return t


def wait(timeout: float | None = None) -> None:
    """Join every warming / building thread started so far."""
    with _LOCK:
        threads = [t for ts in _THREADS.values() for t in ts] + list(_EXTRA)
        _EXTRA.clear()
    for t in threads:
        t.join(timeout)


def _run(dev: torch.device, groups) -> None:
    try:
        with torch.cuda.device(dev):
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                for grp in groups:
                    grp(dev)
            s.synchronize()
    except Exception as e:      # best effort: the stage's own first call stays cold
        errors.append(("prewarm", repr(e)))
        log.debug("prewarm stopped: %s", e)


def _consensus_chain(dev: torch.device) -> None:
    """The k-selection / consensus chain (api.cNMF._consensus) on a toy problem: 24
    "spectra" of 16 genes in 3 clusters."""
    from ..models.consensus import (cluster_medians, kmeans, l2_normalize_rows, local_density,
                                    pairwise_distances, silhouette)

    g = torch.Generator().manual_seed(0)
    S = (torch.rand((24, 16), generator=g, dtype=torch.float64) + 0.1).to(dev)
    L2 = l2_normalize_rows(S)
    d = pairwise_distances(L2)
    local_density(d, 3)
    lab = kmeans(L2, 3, n_init=1, backend="device", device_restart_factor=1)
    silhouette(d, lab)
    cluster_medians(L2, lab, sorted(set(np.asarray(lab).tolist())))


def _library_gemms(dev: torch.device) -> None:
    """The refit's and the prediction error's K x K Grams (segsum.hip small_gram, f32 and
    f64) and the dense-input numerator products (library GEMMs: a resident dense X)."""
    from .. import ops

    g = torch.Generator().manual_seed(1)
    W = torch.rand((3, 16), generator=g).to(dev)
    X = torch.rand((40, 16), generator=g).to(dev)
    _ = ops.small_gram(W, rows_are_points=False)
    _ = X @ W.t()
    U = torch.rand((40, 3), generator=g, dtype=torch.float64).to(dev)
    S3 = torch.rand((3, 16), generator=g, dtype=torch.float64).to(dev)
    q = (ops.small_gram(U) * ops.small_gram(S3, rows_are_points=False)).sum()
    xb = X.to(torch.float64)
    q = q + ((U.t() @ xb) * S3).sum() + (xb * xb).sum()
    float(q)


def _elementwise(dev: torch.device) -> None:
    """Elementwise / reduction / sort kernels of those stages."""
    g = torch.Generator().manual_seed(2)
    t = torch.rand(64, generator=g).to(dev)
    _ = torch.clamp(t, min=0.0), torch.minimum(t, t), torch.maximum(t, t), t.pow(2)
    _ = torch.where(t > 0.5, t, torch.zeros_like(t)), torch.nan_to_num(t), t.sqrt()
    _ = t.var(), t.min(), t.any(), torch.argmin(t), torch.cumsum(t, 0), t.sort()
    _ = torch.unique(t.round()), torch.searchsorted(t.sort().values, t)
    t.sum().item()


_GROUPS = (_consensus_chain, _library_gemms, _elementwise)

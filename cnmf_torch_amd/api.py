"""The ``cNMF`` pipeline object (L5 API; cnmf.py:390-1384).

Same constructor, stage methods, arguments, artifact names and on-disk layout as the
reference, on the MI355X-native engine:

* ``factorize`` groups the worker's ledger rows by K and solves each group as ONE
  replicate batch on the device (models/nmf.py) instead of one replicate at a time,
  still writing one ``spectra.k_%d.iter_%d.df.npz`` per replicate (atomic writes).
* ``refit_usage`` / ``refit_spectra`` use the fused on-device refit (models/refit.py).
* ``consensus`` runs the pairwise distances, density filter, medians and silhouette on
  the device.  KMeans: ``kmeans_backend='auto'`` (the default) runs the batched device
  k-means (k-means++ + Lloyd, 4 x n_init restarts, best inertia; its own RNG stream, so
  the partition can differ from sklearn's where two partitions have close inertia) when
  the spectra are on a GPU, and sklearn on the CPU; ``'sklearn'`` is the reference's
  exact ``KMeans(n_clusters=k, n_init=10, random_state=1)`` (cnmf.py:1082) on any device
  -- the choice for bit-level parity with the reference.
* multi-worker / multi-GPU: ``factorize(worker_i, total_workers)`` keeps the
  round-robin ledger sharding of cnmf.py:53-54 (CLI ``--worker-index`` restored);
  ``cnmf_torch_amd.parallel`` launches one rank per GPU over torch.distributed.
"""
from __future__ import annotations

import concurrent.futures as cf
import datetime
import errno
import itertools
import json
import os
import shutil
import sys
import threading
import time
import uuid
import warnings

import numpy as np
import pandas as pd
import scipy.sparse as sp
import torch
from torch.utils.weak import WeakIdKeyDictionary

from .models.consensus import (cluster_medians, kmeans, l2_normalize_rows, local_density,
                               pairwise_distances, silhouette)
from .models.hvg import (compute_tpm, exact_mean_var, get_highvar_genes,
                         get_highvar_genes_sparse, get_mean_var)
from .models.nmf import NMFBatchSolver, NMFOptions
from . import ops
from .models.ols import efficient_ols_all_cols
from .models.pp import scale as pp_scale
from .models.refit import col_block, fit_H_online, fit_spectra_online, gene_blocks
from .ops import sparse as sops
from .parallel.ledger import worker_filter
from .utils.anndata_lite import AnnData
from .utils import resident
from .utils.transfer import to_host
from .utils.h5ad import read_h5ad, write_h5ad, write_h5ad_row_blocks
from .utils.io import (check_dir_exists, dump_yaml, load_df_from_npz, load_yaml, read_10x_mtx,
                       read_any, read_counts_table, read_spectra_batch, save_arrays_npz_digest,
                       save_df_to_npz,
                       save_df_to_text, NPZ_TMP_LEVEL, write_spectra_batch, write_text_atomic)
from .utils.log import get_logger
from .utils.timing import StageTimer, append_jsonl_many, read_jsonl

log = get_logger("cnmf_torch_amd.api")


def _sha256(path: str) -> str:
    import hashlib

    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()

_PATHS = {
    "normalized_counts": ("tmp", "{name}.norm_counts.h5ad"),
    "nmf_replicate_parameters": ("tmp", "{name}.nmf_params.df.npz"),
    "nmf_run_parameters": ("tmp", "{name}.nmf_idvrun_params.yaml"),
    "nmf_genes_list": ("top", "{name}.overdispersed_genes.txt"),
    "tpm": ("tmp", "{name}.tpm.h5ad"),
    "tpm_stats": ("tmp", "{name}.tpm_stats.df.npz"),
    "iter_spectra": ("tmp", "{name}.spectra.k_%d.iter_%d.df.npz"),
    "iter_usages": ("tmp", "{name}.usages.k_%d.iter_%d.df.npz"),
    "merged_spectra": ("tmp", "{name}.spectra.k_%d.merged.df.npz"),
    "local_density_cache": ("tmp", "{name}.local_density_cache.k_%d.merged.df.npz"),
    "consensus_spectra": ("tmp", "{name}.spectra.k_%d.dt_%s.consensus.df.npz"),
    "consensus_spectra__txt": ("top", "{name}.spectra.k_%d.dt_%s.consensus.txt"),
    "consensus_usages": ("tmp", "{name}.usages.k_%d.dt_%s.consensus.df.npz"),
    "consensus_usages__txt": ("top", "{name}.usages.k_%d.dt_%s.consensus.txt"),
    "consensus_stats": ("tmp", "{name}.stats.k_%d.dt_%s.df.npz"),
    "clustering_plot": ("top", "{name}.clustering.k_%d.dt_%s.png"),
    "gene_spectra_score": ("tmp", "{name}.gene_spectra_score.k_%d.dt_%s.df.npz"),
    "gene_spectra_score__txt": ("top", "{name}.gene_spectra_score.k_%d.dt_%s.txt"),
    "gene_spectra_tpm": ("tmp", "{name}.gene_spectra_tpm.k_%d.dt_%s.df.npz"),
    "gene_spectra_tpm__txt": ("top", "{name}.gene_spectra_tpm.k_%d.dt_%s.txt"),
    "starcat_spectra": ("tmp", "{name}.starcat_spectra.k_%d.dt_%s.df.npz"),
    "starcat_spectra__txt": ("top", "{name}.starcat_spectra.k_%d.dt_%s.txt"),
    "k_selection_plot": ("top", "{name}.k_selection.png"),
    "k_selection_stats": ("top", "{name}.k_selection_stats.df.npz"),
    # additions (not in the reference): per-replicate solver records
    "replicate_log": ("tmp", "{name}.replicates.jsonl"),
    "replicate_manifest": ("tmp", "{name}.spectra_manifest.jsonl"),
}

# nmf-torch run_nmf defaults that the reference leaves implicit
_SOLVER_DEFAULTS = dict(fp_precision="float", online_max_pass=20, online_h_tol=0.05,
                        online_w_tol=0.05, batch_max_iter=500, batch_hals_tol=0.05,
                        batch_hals_max_iter=200)


def _dt_str(density_threshold) -> str:
    return str(density_threshold).replace(".", "_")


def gpu_max_rank(beta_loss="frobenius", algo="mu") -> int | None:
    """Largest K the native MI355X kernels factorise (None: no limit), as
    models.nmf_base.kernel_max_rank: Frobenius MU and the beta-divergences any K
    (register-tiled kernels to 128 / 64 / 56, the rank-general paths beyond), HALS 512,
    'bpp' any K (torch linear algebra)."""
    from .models.nmf import beta_value, kernel_max_rank

    return kernel_max_rank(beta_value(beta_loss), algo)


def check_gpu_ranks(components, beta_loss="frobenius", algo="mu", use_gpu=True) -> list:
    """Say at once -- at ``prepare``, before any work -- which ranks the native GPU kernels
    do not cover (the reference's ``-k`` is unbounded, cnmf.py:1417).  Those replicates
    are routed to the eager PyTorch ops on the same GPU (NMFBatchSolver.run, ops.eager_ops)
    instead of failing the job.  Returns the uncovered ranks."""
    if not use_gpu or not torch.cuda.is_available():
        return []
    ks = sorted({int(k) for k in np.atleast_1d(components)})
    kmax = gpu_max_rank(beta_loss, algo)
    over = [k for k in ks if kmax is not None and k > kmax]
    if over:
        msg = (f"K={over}: the native gfx950 kernels factorise K <= {kmax} "
               f"(beta_loss={beta_loss!r}, algo={algo!r}); these ranks run the eager "
               "PyTorch ops on the GPU (slower)")
        warnings.warn(msg, RuntimeWarning, stacklevel=2)
        log.warning(msg)
    return over


def _gpu_visible() -> bool:
    """torch.cuda.is_available(), asked once per process (utils.gpu)."""
    from .utils.gpu import visible

    return visible()


def _device(use_gpu: bool, device=None) -> torch.device:
    """Explicit ``device`` > $CNMF_DEVICE > the local GPU when one is visible > CPU.

    The reference's ``use_gpu`` (default False) selected nmf-torch's CUDA path; this
    framework is GPU-first, so a visible MI355X is used unless told otherwise.
    ``use_gpu=True`` without a GPU falls back to the CPU with a warning (nmf-torch
    falls back silently)."""
    if device is None:
        device = os.environ.get("CNMF_DEVICE") or None
    if device is not None:
        return torch.device(device)
    if _gpu_visible():
        return torch.device("cuda", torch.cuda.current_device())
    if use_gpu:
        warnings.warn("use_gpu=True but no GPU is visible; running on the CPU")
    return torch.device("cpu")


def _device_csr(X, dev: torch.device):
    """A sparse host matrix uploaded once as a device CSR when running on a GPU, else None."""
    if dev.type != "cuda" or not sp.issparse(X):
        return None
    return sops.DeviceCSR.from_scipy(X, device=dev)


def _device_csr_cached(adata, dev: torch.device):
    """:func:`_device_csr` of ``adata.X``, kept on the AnnData (keyed on X's identity and
    the device) so repeated consensus calls on one TPM upload it once."""
    if dev.type != "cuda" or not sp.issparse(adata.X):
        return None
    cache = adata.__dict__.setdefault("_cnmf_device_csr", {})
    key = (str(dev), id(adata.X))
    if key not in cache:
        cache.clear()
        cache[key] = _device_csr(adata.X, dev)
    return cache[key]


def _norm_counts_dense_device(counts, genes, guard_zero_std: bool, dev) -> AnnData:
    """get_norm_counts for a dense count matrix on the GPU (cnmf.py:670-681): the HVG
    column gather, the float64 cast and the unit-variance scaling run on the device; one
    H2D of the counts and one D2H of the float64 result.  ``guard_zero_std`` selects
    scanpy's scale (E[x^2] - E[x]^2, ddof=1, std 0 -> 1; used when the TPM is sparse)
    over numpy's ``X / X.std(ddof=1)`` (two-pass, no guard)."""
    T, cols = _norm_counts_tensor(counts, genes, guard_zero_std, dev)
    out = AnnData(X=to_host(T), obs=counts.obs, var=counts.var.iloc[cols],
                  obsm=dict(counts.obsm), uns=dict(counts.uns))
    out.uns["_scaled_on_device"] = True
    return out


def _save_norm_counts_streamed(path: str, counts, T: torch.Tensor, cols, rows: int = 16384):
    """Write the device-resident float64 norm counts ``T`` as the h5ad of
    get_norm_counts(...) without a whole-matrix host copy: row blocks go D2H into two
    pinned staging buffers on a copy stream while the previous block is written, so the
    copy overlaps the file write (500k x 2000 float64 = 8 GB: the whole-matrix .cpu() and
    the numpy NaN / zero-row passes took ~1.3 s of prepare, profiles/r3ac_*)."""
    n, G = T.shape
    rows = max(1, min(rows, n))
    bufs = [torch.empty((rows, G), dtype=T.dtype, pin_memory=True) for _ in range(2)]
    evs = [torch.cuda.Event() for _ in range(2)]
    cs = torch.cuda.Stream(T.device)
    cs.wait_stream(torch.cuda.current_stream(T.device))

    def issue(i):
        a = i * rows
        b = min(n, a + rows)
        with torch.cuda.stream(cs):
            bufs[i % 2][:b - a].copy_(T[a:b], non_blocking=True)
            evs[i % 2].record(cs)
        return b - a

    nblk = -(-n // rows)

    def blocks():
        m = issue(0)
        for i in range(nblk):
            evs[i % 2].synchronize()
            nxt = issue(i + 1) if i + 1 < nblk else 0
            yield None, bufs[i % 2][:m].numpy()
            m = nxt

    try:
        write_h5ad_row_blocks(path, n, counts.var.iloc[cols], blocks(), sparse=False,
                              dtype=np.float64, obs=counts.obs, obsm=dict(counts.obsm),
                              uns=dict(counts.uns))
    finally:
        cs.synchronize()   # no copy may still target a staging buffer (error path)


def _norm_counts_tensor(counts, genes, guard_zero_std: bool, dev):
    """(device float64 norm counts, gene column indices) of a dense count matrix."""
    cols = counts.var.index.get_indexer(list(genes))
    if (cols < 0).any():
        raise KeyError(f"genes missing from the counts: {list(np.array(genes)[cols < 0][:5])}")
    T = torch.from_numpy(np.ascontiguousarray(counts.X)).to(dev)
    T = T.index_select(1, torch.as_tensor(cols, device=dev)).to(torch.float64)
    n = T.shape[0]
    ex = exact_mean_var(T, 1)        # exact moments on the device (models.hvg)
    if ex is not None:
        std = torch.from_numpy(np.sqrt(ex[1])).to(dev)
        if guard_zero_std:
            std[std == 0] = 1.0
    elif guard_zero_std:
        mean = T.mean(dim=0)
        var = (T * T).mean(dim=0) - mean * mean
        if n > 1:
            var *= n / (n - 1)
        std = torch.sqrt(var)
        std[std == 0] = 1.0
    else:
        std = T.std(dim=0, unbiased=True)
    T /= std
    return T, cols


def _resident_X(adata, dev: torch.device):
    """``adata.X`` on the device, uploaded once per AnnData object and device and reused
    by every K of k_selection_plot (refit numerators, prediction error): a DeviceCSR for
    sparse X, a float32 tensor for dense X; the host matrix itself on the CPU.  The
    cached copy is keyed on the identity of ``adata.X``; an AnnData from
    :meth:`cNMF._read_norm_counts` arrives with X = None and its resident mirror preset."""
    cache = adata.__dict__.setdefault("_cnmf_device_X", {})
    key = (str(dev), id(adata.X))
    if key in cache:
        return cache[key]
    if dev.type != "cuda":
        return adata.X
    if key not in cache:
        cache.clear()
        X = adata.X
        cache[key] = (_device_csr(X, dev) if sp.issparse(X)
                      else torch.as_tensor(np.asarray(X, dtype=np.float32)).to(dev))
    return cache[key]


# cooperative (co-resident, spinning) solves of concurrent k-selection threads
_COOP_LOCK = threading.RLock()
# k-selection worker threads (one HIP stream each; 8 measured the same as 4: profiles/r5zo_*)
_KSEL_THREADS = 4

# ||X||^2 of a device-resident X (api._prediction_error), weakly keyed by the tensor's
# identity (a WeakKeyDictionary compares tensor keys with Tensor.__eq__, which raises)
_XSQ = WeakIdKeyDictionary()


def sops_predict(X, U, S):
    from . import ops as _ops

    return _ops.predict_err_terms(X, U, S)


def _load_npz_arrays(fn: str):
    """(data, index, columns) arrays of a .df.npz without building a DataFrame."""
    try:
        with np.load(fn, allow_pickle=False) as f:
            return f["data"], f["index"], f["columns"]
    except ValueError:
        df = load_df_from_npz(fn)          # object arrays from the original cnmf
        return df.values, df.index.values, df.columns.values


def _dense32(X) -> np.ndarray:
    if sp.issparse(X):
        return X.astype(np.float32).toarray()
    return np.asarray(X, dtype=np.float32)


class cNMF:
    """Consensus NMF pipeline (cnmf.py:390)."""

    def __init__(self, output_dir: str = ".", name: str | None = None):
        self.output_dir = output_dir
        if name is None:
            now = datetime.datetime.now()
            name = "%s_%s" % (now.strftime("%Y_%m_%d"), uuid.uuid4().hex[:6])
        self.name = name
        self.paths = None
        self.timer = StageTimer()
        self._initialize_dirs()

    # ------------------------------------------------------------------ paths
    def _initialize_dirs(self):
        if self.paths is not None:
            return
        top = os.path.join(self.output_dir, self.name)
        tmp = os.path.join(top, "cnmf_tmp")
        check_dir_exists(self.output_dir)
        check_dir_exists(top)
        check_dir_exists(tmp)
        self.paths = {k: os.path.join(tmp if where == "tmp" else top, pat.format(name=self.name))
                      for k, (where, pat) in _PATHS.items()}

    # ------------------------------------------------------------------ prepare
    def prepare(self, counts_fn, components, n_iter=100, densify=False, tpm_fn=None, seed=None,
                beta_loss="frobenius", num_highvar_genes=2000, genes_file=None, alpha_usage=0.0,
                alpha_spectra=0.0, init="random", total_workers=-1, use_gpu=False,
                batch_size=5000, max_NMF_iter=1000, algo="mu", mode="online", comm=None,
                prewarm=True):
        """Load counts, select over-dispersed genes, variance-normalise, write the
        replicate ledger (cnmf.py:458-596).  ``algo``/``mode`` are additions (defaults =
        the reference's hard-coded 'mu'/'online').  With a multi-rank ``comm`` the cells
        are sharded over the ranks and the per-gene statistics are all-reduced
        (:meth:`_prepare_sharded`).

        ``prewarm`` (GPU): while this stage runs, a background thread makes the first
        launches of the k-selection / consensus kernels in this process
        (utils.prewarm), so those stages do not pay HIP's first-use code loading later
        in the same process (joined before returning), and the figure process starts
        (utils.plotting.prestart).  The CLI, whose later stages are other processes,
        turns it off."""
        check_gpu_ranks(components, beta_loss, algo, use_gpu)
        if comm is not None and comm.world_size > 1:
            return self._prepare_sharded(
                comm, counts_fn, components, n_iter=n_iter, densify=densify, tpm_fn=tpm_fn,
                seed=seed, beta_loss=beta_loss, num_highvar_genes=num_highvar_genes,
                genes_file=genes_file, alpha_usage=alpha_usage, alpha_spectra=alpha_spectra,
                init=init, total_workers=total_workers, use_gpu=use_gpu, batch_size=batch_size,
                max_NMF_iter=max_NMF_iter, algo=algo, mode=mode)
        warm = prewarm and _device(False).type == "cuda"
        if warm:
            from .utils import prewarm as _prewarm
            from .utils.plotting import prestart

            # one thread per group: the code-object loads overlap (0.24 vs 0.53 s on one
            # thread, profiles/r5zj_*), inside prepare's own host work once the planes
            # build is factorize's again (_prebuild_planes)
            _prewarm.start(_device(False), parallel=True)
            self._prebuild = True
            # and the figure process (matplotlib's import) a stage earlier than factorize
            # would start it: with the later stages warm it is the pipeline's last wait
            prestart()
        try:
            self._prepare_local(counts_fn, components, n_iter, densify, tpm_fn, seed,
                                beta_loss, num_highvar_genes, genes_file, alpha_usage,
                                alpha_spectra, init, total_workers, use_gpu, batch_size,
                                max_NMF_iter, algo, mode)
        finally:
            self._prebuild = False
            if warm:
                _prewarm.wait()

    def _prepare_local(self, counts_fn, components, n_iter, densify, tpm_fn, seed, beta_loss,
                       num_highvar_genes, genes_file, alpha_usage, alpha_spectra, init,
                       total_workers, use_gpu, batch_size, max_NMF_iter, algo, mode):
        """Single-process prepare (see prepare).  An .h5ad ``tpm_fn`` is copied on a
        background thread while the rest of the stage runs on the object read from the
        source (joined before the stage ends, also on an error) -- the copy of the 5 GB
        TP10K file was 0.5 s of the 500k-cell prepare (profiles/r4h_*)."""
        copies = []
        with self.timer("prepare"):
            try:
                input_counts = read_any(counts_fn, densify)
                if sp.issparse(input_counts.X) and densify:
                    input_counts.X = np.array(input_counts.X.todense())

                if tpm_fn is None:
                    tpm = compute_tpm(input_counts)
                    write_h5ad(self.paths["tpm"], tpm)
                elif tpm_fn.endswith(".mtx") or tpm_fn.endswith(".mtx.gz"):
                    tpm = read_10x_mtx(os.path.dirname(tpm_fn))
                    write_h5ad(self.paths["tpm"], tpm)
                elif tpm_fn.endswith(".h5ad"):
                    pool = cf.ThreadPoolExecutor(1, thread_name_prefix="cnmf-tpm-copy")
                    copies.append(pool.submit(shutil.copyfile, tpm_fn, self.paths["tpm"]))
                    pool.shutdown(wait=False)
                    tpm = read_h5ad(tpm_fn)
                else:
                    tpm = read_counts_table(tpm_fn, densify)
                    write_h5ad(self.paths["tpm"], tpm)
                if not copies and _device(False).type == "cuda":
                    # consensus in this process takes this object instead of re-reading the
                    # file (utils.resident: only while the file is unchanged)
                    resident.remember(self.paths["tpm"], "adata", tpm)

                # exact moments on the host matrix (models.hvg.exact_mean_var): the same bits
                # as the cell-sharded prepare's all-reduced digits (_prepare_sharded)
                ex = exact_mean_var(tpm.X, 0)
                if ex is not None:
                    gene_tpm_mean, gene_tpm_var = ex
                    if tpm.X.dtype == np.float32:   # sklearn keeps float32 statistics
                        gene_tpm_mean = gene_tpm_mean.astype(np.float32)
                        gene_tpm_var = gene_tpm_var.astype(np.float32)
                    gene_tpm_std = gene_tpm_var ** 0.5
                elif sp.issparse(tpm.X):
                    dT = _device_csr(tpm.X, _device(use_gpu))
                    gene_tpm_mean, gene_tpm_var = get_mean_var(dT if dT is not None else tpm.X)
                    del dT
                    gene_tpm_std = gene_tpm_var ** 0.5
                else:
                    gene_tpm_mean = np.array(tpm.X.mean(axis=0)).reshape(-1)
                    gene_tpm_std = np.array(tpm.X.std(axis=0, ddof=0)).reshape(-1)
                stats = pd.DataFrame([gene_tpm_mean, gene_tpm_std], index=["__mean", "__std"],
                                     columns=tpm.var.index).T
                save_df_to_npz(stats, self.paths["tpm_stats"])

                highvargenes = None
                if genes_file is not None:
                    with open(genes_file) as fh:
                        highvargenes = fh.read().rstrip().split("\n")

                dev = _device(False)
                if not sp.issparse(input_counts.X) and dev.type == "cuda":
                    # dense counts on the GPU: scaled, checked and streamed to the h5ad from
                    # the device (same file and messages as get_norm_counts + save)
                    genes = self._hvg_filter(tpm, highvargenes, num_highvar_genes)
                    T, cols = _norm_counts_tensor(input_counts, genes, sp.issparse(tpm.X), dev)
                    self._check_norm_counts(T, input_counts.obs.index, genes)
                    self._initialize_dirs()
                    _save_norm_counts_streamed(self.paths["normalized_counts"], input_counts, T,
                                               cols)
                    # factorize / consensus in this process read the device copy, not the file
                    # (utils.resident; the float32 cast is the one they apply to the file's data)
                    resident.remember(self.paths["normalized_counts"], "X32", T.to(torch.float32))
                    del T
                    self._prebuild_planes(dev)
                else:
                    norm_counts = self.get_norm_counts(input_counts, tpm,
                                                       num_highvar_genes=num_highvar_genes,
                                                       high_variance_genes_filter=highvargenes)
                    self.save_norm_counts(norm_counts)
                    if dev.type == "cuda" and resident.wanted(norm_counts.X):
                        # the float32 device matrix factorize would build from the file
                        # (a sparse file: only factorize densifies it; consensus reads the
                        # file's CSR, see _read_norm_counts)
                        tag = "X32_factorize" if sp.issparse(norm_counts.X) else "X32"
                        resident.remember(self.paths["normalized_counts"], tag,
                                          torch.from_numpy(_dense32(norm_counts.X)).to(dev))
                        self._prebuild_planes(dev)
                replicate_params, run_params = self.get_nmf_iter_params(
                    ks=components, n_iter=n_iter, random_state_seed=seed, beta_loss=beta_loss,
                    alpha_usage=alpha_usage, alpha_spectra=alpha_spectra, init=init,
                    total_workers=total_workers, use_gpu=use_gpu, batch_size=batch_size,
                    max_iter=max_NMF_iter, algo=algo, mode=mode)
                self.save_nmf_iter_params(replicate_params, run_params)
                for c in copies:
                    c.result()
            except BaseException:
                for c in copies:        # no copy left running behind the error
                    c.exception()
                raise
        if copies and _device(False).type == "cuda":
            # (after the copy: the mirror is keyed on the finished file's identity)
            resident.remember(self.paths["tpm"], "adata", tpm)

    def _prebuild_planes(self, dev) -> None:
        """Opt-in (CNMF_PREBUILD_PLANES=1, with prepare's prewarm on): build the resident
        matrix's split-GEMM planes on a background thread (models.nmf_base.planes_ahead)
        for factorize in this process.  Off by default: factorize builds and times its
        own planes (the build is factorize work, not prepare's)."""
        if not getattr(self, "_prebuild", False) or \
                os.environ.get("CNMF_PREBUILD_PLANES", "0") != "1":
            return
        path = self.paths["normalized_counts"]
        X = resident.recall(path, "X32")
        if X is None:
            X = resident.recall(path, "X32_factorize")
        if X is None or X.device != dev:
            return
        from .models.nmf_base import planes_ahead
        from .utils import prewarm as _prewarm

        X_ready = torch.cuda.Event()
        X_ready.record()            # the mirror's upload, on this thread's stream

        def build():
            torch.cuda.current_stream().wait_event(X_ready)
            planes_ahead(X)

        _prewarm.run(dev, build)

    def _prepare_sharded(self, comm, counts_fn, components, n_iter, densify, tpm_fn, seed,
                         beta_loss, num_highvar_genes, genes_file, alpha_usage, alpha_spectra,
                         init, total_workers, use_gpu, batch_size, max_NMF_iter, algo, mode):
        """Cell-sharded prepare: rank r holds a contiguous block of
        cells (partial h5ad read), computes its TPM rows, and the per-gene statistics --
        TPM mean/variance for tpm_stats and the over-dispersion model, the ddof=1 std of
        the HVG counts for the unit-variance scaling -- are combined across ranks by
        all-reduces (two-pass: global mean first, then centred sums of squares, so the
        variances equal the single-process ones to summation order).  Rank 0 writes the
        artifacts of the single-process prepare, receiving the other ranks' row blocks
        one rank at a time (point-to-point) straight into the h5ad datasets: it never
        holds more than its own block and one peer's (h5ad.write_h5ad_row_blocks)."""
        import pickle

        from .parallel.runner import row_block
        from .utils.io import read_rows_any

        rank, world = comm.rank, comm.world_size
        # bound of every point-to-point message of the row-block hand-over (bytes)
        cb = int(os.environ.get("CNMF_PREPARE_CHUNK_BYTES", str(1 << 30)))
        with self.timer("prepare"):
            if tpm_fn is not None:
                raise NotImplementedError("sharded prepare computes the TPM itself "
                                          "(tpm_fn: run prepare on one rank)")
            # only this rank's cells are read (h5ad / 10x mtx / DataFrame npz / TSV)
            counts, _, _ = read_rows_any(counts_fn, lambda n: row_block(n, rank, world),
                                         densify)
            if sp.issparse(counts.X) and densify:
                counts.X = np.asarray(counts.X.todense())
            sparse_in = sp.issparse(counts.X)
            tpm = compute_tpm(counts)

            def col_sum(M):
                return np.asarray(M.sum(axis=0), dtype=np.float64).reshape(-1)

            # the per-gene moments of this rank's block run on its GPU when there is one
            # (exact integer digits either way: the same statistics bit for bit)
            sdev = None
            if torch.cuda.is_available() and ops.native_available():
                sdev = torch.device("cuda", torch.cuda.current_device())

            def mean_var(M, ddof):
                """Global column mean / variance of the row-sharded M: the exact integer
                moments all-reduced (models.hvg.exact_mean_var -- the single-process
                prepare's statistics, bit for bit), else the float64 two-pass."""
                ex = exact_mean_var(M, ddof, comm, device=sdev)
                if ex is not None:
                    return ex
                n = comm.allreduce_scalar(float(M.shape[0]))
                s1 = torch.from_numpy(col_sum(M))
                comm.allreduce_(s1)
                mean = s1.numpy() / max(n, 1.0)
                if sp.issparse(M):
                    Mc = M.tocsc() if not sp.isspmatrix_csc(M) else M
                    d = Mc.data.astype(np.float64) - np.repeat(mean, np.diff(Mc.indptr))
                    nnz = np.diff(Mc.indptr).astype(np.float64)
                    m2 = np.bincount(np.repeat(np.arange(M.shape[1]), np.diff(Mc.indptr)),
                                     weights=d * d, minlength=M.shape[1])
                    m2 = m2 + (M.shape[0] - nnz) * mean * mean
                else:
                    d = np.asarray(M, dtype=np.float64) - mean
                    m2 = (d * d).sum(axis=0)
                m2 = torch.from_numpy(np.ascontiguousarray(m2, dtype=np.float64))
                comm.allreduce_(m2)
                return mean, m2.numpy() / max(n - ddof, 1.0)

            gene_tpm_mean, gene_tpm_var = mean_var(tpm.X, 0)
            hv_mean, hv_var = gene_tpm_mean, gene_tpm_var
            if tpm.X.dtype == np.float32:     # sklearn keeps float32 statistics
                gene_tpm_mean = gene_tpm_mean.astype(np.float32)
                gene_tpm_var = gene_tpm_var.astype(np.float32)
                if sparse_in:     # get_highvar_genes_sparse sees get_mean_var's float32
                    hv_mean = gene_tpm_mean.astype(np.float64)
                    hv_var = gene_tpm_var.astype(np.float64)
            gene_tpm_std = gene_tpm_var ** 0.5
            stats = pd.DataFrame([gene_tpm_mean, gene_tpm_std], index=["__mean", "__std"],
                                 columns=tpm.var.index).T
            if genes_file is not None:
                with open(genes_file) as fh:
                    hvgs = fh.read().rstrip().split("\n")
            else:
                from .models.hvg import _fano_model

                gstats, _ = _fano_model(pd.Series(hv_mean), pd.Series(hv_var),
                                        None, 0.5, num_highvar_genes)
                hvgs = list(tpm.var.index[gstats.high_var.values])
            cols = counts.var.index.get_indexer(hvgs)
            if (cols < 0).any():
                raise KeyError(f"genes missing from the counts: {list(np.array(hvgs)[cols < 0][:5])}")
            Xh = counts.X[:, cols]
            Xh = Xh.astype(np.float64) if sp.issparse(Xh) else np.asarray(Xh, dtype=np.float64)
            _, hv_cvar = mean_var(Xh, 1)
            std = np.sqrt(hv_cvar)
            if sparse_in:          # scanpy scale(zero_center=False): std 0 -> 1
                std[std == 0] = 1.0
                Xh = sp.csr_matrix(Xh)
                Xh.data = Xh.data / std[Xh.indices]
            else:                  # dense reference path: X / X.std(ddof=1), no guard
                with np.errstate(divide="ignore", invalid="ignore"):
                    Xh = Xh / std
            zero = np.asarray(Xh.sum(axis=1)).reshape(-1) == 0
            n_zero = int(comm.allreduce_scalar(float(zero.sum())))
            if n_zero > 0:
                ex = counts.obs.index[zero][:4]
                raise Exception(
                    "Error: %d cells have zero counts of overdispersed genes. E.g. %s. Filter "
                    "those cells and re-run or adjust the number of overdispersed genes. "
                    "Quitting!" % (n_zero, ", ".join(ex)))
            from .utils.h5ad import write_h5ad_row_blocks

            def nnz(M):
                return int(M.nnz) if sp.issparse(M) else 0
            meta = comm.all_gather_object((int(tpm.X.shape[0]), nnz(tpm.X), nnz(Xh)))
            if rank == 0:
                self._initialize_dirs()
            n_tot = sum(m_[0] for m_ in meta)

            def send_block(obs, M):
                """A peer's row block to rank 0: arrays in messages of <= cb bytes."""
                comm.send_array(np.frombuffer(pickle.dumps(obs), dtype=np.uint8), 0, cb)
                if sp.issparse(M):
                    M = sp.csr_matrix(M)
                    for arr in (M.data, M.indices, M.indptr.astype(np.int64)):
                        comm.send_array(arr, 0, cb)
                else:
                    comm.send_array(np.asarray(M), 0, cb)

            def recv_block(src, G_):
                obs = pickle.loads(comm.recv_array(src).tobytes())
                if sparse_in:
                    data, ind, ptr = (comm.recv_array(src) for _ in range(3))
                    return obs, sp.csr_matrix((data, ind, ptr), shape=(len(obs), G_))
                return obs, comm.recv_array(src)

            for which, local, total_nnz, path, var in (
                    (0, tpm.X, sum(m_[1] for m_ in meta), self.paths["tpm"], tpm.var),
                    (1, Xh, sum(m_[2] for m_ in meta), self.paths["normalized_counts"],
                     counts.var.iloc[cols])):
                failed = None
                if rank == 0:
                    def blocks(local=local, G_=len(var)):
                        yield counts.obs, local
                        for src in range(1, world):       # one peer block at a time
                            yield recv_block(src, G_)
                    gen = blocks()
                    idx_dt = np.int64 if total_nnz >= 2 ** 31 else np.int32
                    try:
                        write_h5ad_row_blocks(path, n_tot, var, gen, sparse_in, local.dtype,
                                              total_nnz, idx_dt)
                    except Exception as e:       # noqa: BLE001 -- re-raised below
                        failed = e
                        for _ in gen:    # keep receiving: no peer is left blocked in a send
                            pass
                else:
                    send_block(counts.obs, local)
                # rank 0 tells every peer whether the file was written: a writer failure
                # fails the stage on every rank instead of leaving peers in a barrier
                st = torch.tensor([0 if failed is None else 1], dtype=torch.int64,
                                  device=comm._dev() if hasattr(comm, "_dev") else "cpu")
                comm.broadcast_(st, src=0)
                if failed is not None:
                    raise failed
                if int(st.item()) != 0:
                    raise RuntimeError(f"sharded prepare: rank 0 failed to write {path}")
            if rank == 0:
                save_df_to_npz(stats, self.paths["tpm_stats"])
                write_text_atomic(self.paths["nmf_genes_list"], "\n".join(hvgs))
                replicate_params, run_params = self.get_nmf_iter_params(
                    ks=components, n_iter=n_iter, random_state_seed=seed, beta_loss=beta_loss,
                    alpha_usage=alpha_usage, alpha_spectra=alpha_spectra, init=init,
                    total_workers=total_workers, use_gpu=use_gpu, batch_size=batch_size,
                    max_iter=max_NMF_iter, algo=algo, mode=mode)
                self.save_nmf_iter_params(replicate_params, run_params)
            comm.barrier()

    @staticmethod
    def _hvg_filter(tpm, high_variance_genes_filter, num_highvar_genes):
        """The over-dispersed genes (fano model on the TPM) unless a list is given."""
        if high_variance_genes_filter is None:
            if sp.issparse(tpm.X):
                gstats, _ = get_highvar_genes_sparse(tpm.X, numgenes=num_highvar_genes)
            else:
                gstats, _ = get_highvar_genes(np.array(tpm.X), numgenes=num_highvar_genes)
            high_variance_genes_filter = list(tpm.var.index[gstats.high_var.values])
        return high_variance_genes_filter

    def _check_norm_counts(self, T: torch.Tensor, obs_index, genes) -> None:
        """get_norm_counts's NaN warning and zero-row error on a device tensor, plus the
        genes list file (cnmf.py:683-693)."""
        if bool(torch.isnan(T).any()):
            print("Warning NaNs in normalized counts matrix")
        write_text_atomic(self.paths["nmf_genes_list"], "\n".join(genes))
        zerocells = (T.sum(dim=1) == 0).cpu().numpy()
        if zerocells.sum() > 0:
            examples = obs_index[np.ravel(zerocells)]
            raise Exception(
                "Error: %d cells have zero counts of overdispersed genes. E.g. %s. Filter those "
                "cells and re-run or adjust the number of overdispersed genes. Quitting!"
                % (zerocells.sum(), ", ".join(examples[:4])))

    def get_norm_counts(self, counts, tpm, high_variance_genes_filter=None,
                        num_highvar_genes=None):
        """HVG subset of the raw counts, genes scaled to unit variance (cnmf.py:624-693)."""
        high_variance_genes_filter = self._hvg_filter(tpm, high_variance_genes_filter,
                                                      num_highvar_genes)

        dev = _device(False)
        if not sp.issparse(counts.X) and dev.type == "cuda":
            norm_counts = _norm_counts_dense_device(counts, high_variance_genes_filter,
                                                    guard_zero_std=sp.issparse(tpm.X), dev=dev)
        else:
            norm_counts = counts[:, high_variance_genes_filter].copy()
            norm_counts.X = norm_counts.X.astype(np.float64)
        if norm_counts.uns.pop("_scaled_on_device", False):
            if np.isnan(norm_counts.X).sum() > 0:
                print("Warning NaNs in normalized counts matrix")
        elif sp.issparse(tpm.X):
            norm_counts = pp_scale(norm_counts, zero_center=False)
            if np.isnan(norm_counts.X.data).sum() > 0:
                print("Warning NaNs in normalized counts matrix")
        else:
            X = norm_counts.X.toarray() if sp.issparse(norm_counts.X) else norm_counts.X
            ex = exact_mean_var(X, 1)
            std = np.sqrt(ex[1]) if ex is not None else X.std(axis=0, ddof=1)
            with np.errstate(divide="ignore", invalid="ignore"):
                X = X / std
            norm_counts.X = X
            if np.isnan(norm_counts.X).sum().sum() > 0:
                print("Warning NaNs in normalized counts matrix")

        write_text_atomic(self.paths["nmf_genes_list"], "\n".join(high_variance_genes_filter))

        zerocells = np.array(norm_counts.X.sum(axis=1) == 0).reshape(-1)
        if zerocells.sum() > 0:
            examples = norm_counts.obs.index[np.ravel(zerocells)]
            raise Exception(
                "Error: %d cells have zero counts of overdispersed genes. E.g. %s. Filter those "
                "cells and re-run or adjust the number of overdispersed genes. Quitting!"
                % (zerocells.sum(), ", ".join(examples[:4])))
        return norm_counts

    def _read_norm_counts(self, dev: torch.device, factorize: bool = False):
        """The normalized-counts AnnData; when this process wrote the file and still
        holds its device mirror (utils.resident, prepare's GPU path) only obs / var are
        read and X is left None with the mirror preset for :func:`_resident_X`.  The
        mirror of a sparse file serves ``factorize`` only (it densifies X; the other
        stages run the CSR kernels on the file's matrix)."""
        path = self.paths["normalized_counts"]
        Xr = resident.recall(path, "X32")
        if Xr is None and factorize:
            Xr = resident.recall(path, "X32_factorize")
        if Xr is not None and Xr.device == dev:
            from .utils.h5ad import read_h5ad_annotations

            ad = read_h5ad_annotations(path)
            if tuple(ad.shape) == tuple(Xr.shape):
                ad.__dict__["_cnmf_device_X"] = {(str(dev), id(None)): Xr}
                return ad
        return read_h5ad(path)

    def save_norm_counts(self, norm_counts):
        self._initialize_dirs()
        write_h5ad(self.paths["normalized_counts"], norm_counts)

    def get_nmf_iter_params(self, ks, n_iter=100, random_state_seed=None,
                            beta_loss="frobenius", alpha_usage=0.0, alpha_spectra=0.0,
                            init="random", total_workers=-1, use_gpu=False, batch_size=5000,
                            max_iter=1000, algo="mu", mode="online"):
        """Replicate ledger + solver kwargs (cnmf.py:701-777).  Seeds are numpy-legacy
        exact: ``np.random.seed(seed); randint(1, 2**31-1, len(ks)*n_iter)``."""
        if isinstance(ks, (int, np.integer)):
            ks = [ks]
        k_list = sorted(set(list(ks)))
        n_runs = len(ks) * n_iter
        np.random.seed(seed=random_state_seed)
        nmf_seeds = np.random.randint(low=1, high=(2 ** 31) - 1, size=n_runs)
        rows = []
        for i, (k, r) in enumerate(itertools.product(k_list, range(n_iter))):
            done = os.path.exists(self.paths["iter_spectra"] % (k, r))
            rows.append([int(k), int(r), int(nmf_seeds[i]), bool(done)])
        replicate_params = pd.DataFrame(rows, columns=["n_components", "iter", "nmf_seed",
                                                       "completed"])
        n_completed = int(replicate_params["completed"].sum())
        if n_completed > 0:
            warnings.warn(
                f"{n_completed} runs already appear completed. If this is unexpected, consider "
                "re-initializing the cnmf object with a different run name or output directory",
                UserWarning)
        kwargs = dict(alpha_W=alpha_spectra, alpha_H=alpha_usage, l1_ratio_H=0.0,
                      l1_ratio_W=0.0, beta_loss=beta_loss, algo=algo, tol=1e-4, mode=mode,
                      online_chunk_max_iter=max_iter, online_chunk_size=batch_size, init=init,
                      n_jobs=total_workers, use_gpu=use_gpu)
        kwargs.update(_SOLVER_DEFAULTS)
        return replicate_params, kwargs

    def update_nmf_iter_params(self):
        """Refresh the ``completed`` column from the files on disk (cnmf.py:780-795)."""
        kwargs = load_yaml(self.paths["nmf_run_parameters"])
        rp = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        rp["completed"] = [
            os.path.exists(self.paths["iter_spectra"] % (int(k), int(i)))
            for k, i in zip(rp["n_components"], rp["iter"])]
        remaining = int((rp["completed"] == False).sum())  # noqa: E712
        print("{n} NMF runs are currently incomplete".format(n=remaining))
        self.save_nmf_iter_params(rp, kwargs)

    def save_nmf_iter_params(self, replicate_params, run_params):
        self._initialize_dirs()
        save_df_to_npz(replicate_params, self.paths["nmf_replicate_parameters"])
        dump_yaml(run_params, self.paths["nmf_run_parameters"])

    # ------------------------------------------------------------------ factorize
    def _solver_options(self, kwargs: dict, k: int) -> NMFOptions:
        kw = dict(_SOLVER_DEFAULTS)
        kw.update(kwargs)
        return NMFOptions.from_kwargs(k, **kw)

    def _nmf(self, X, nmf_kwargs):
        """One replicate (cnmf.py:805-821): returns (spectra K x G, usages N x K)."""
        k = int(nmf_kwargs["n_components"])
        dev = _device(bool(nmf_kwargs.get("use_gpu", False)))
        Xt = torch.from_numpy(_dense32(X)).to(dev)
        res = NMFBatchSolver(Xt, self._solver_options(nmf_kwargs, k)).run(
            [int(nmf_kwargs["random_state"])])
        return res.spectra(0).cpu().numpy(), res.usages(0).cpu().numpy()

    def factorize(self, worker_i=0, total_workers=1, skip_completed_runs=False, device=None,
                  replicate_batch: int | None = None, save_usages: bool = False, verbose=True):
        """Run this worker's share of the replicate ledger (cnmf.py:839-892).

        Jobs with the same K are solved together in batches of ``replicate_batch``
        replicates (default: all of them that fit the device memory budget).

        Worker 0 also starts the figure process (utils.plotting.prestart): it imports
        matplotlib in the background, so when combine / k_selection_plot / consensus run
        in this same process their closed figures do not wait for that import."""
        if worker_i == 0:
            from .utils.plotting import prestart

            prestart()
        run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        if not skip_completed_runs:
            jobs = list(worker_filter(range(len(run_params)), worker_i, total_workers))
        else:
            done = run_params["completed"].astype(bool).values
            jobs = list(worker_filter(list(run_params.index[~done]), worker_i, total_workers))
        self.factorize_jobs(jobs, worker_label=worker_i, device=device,
                            replicate_batch=replicate_batch, save_usages=save_usages,
                            verbose=verbose, run_params=run_params)

    def factorize_jobs(self, jobs, worker_label=0, device=None, replicate_batch=None,
                       save_usages=False, verbose=True, run_params=None, comm=None,
                       row_range=None, row_segments=None, collect=None):
        """Factorise an explicit list of ledger rows.

        ``collect`` (a dict): also keep every written replicate's spectra in memory,
        ``collect[(k, iter)] = (k x G) float32``, plus ``collect["genes"]`` -- for the
        in-memory gather of parallel.runner.gather_merged_spectra.

        ``comm`` with ``row_segments`` (global [start, stop) row segments, e.g.
        parallel.runner.dp_row_segments) or ``row_range`` (one contiguous block) runs the
        cell-sharded data-parallel solver: this rank holds those rows of norm_counts, the
        sufficient statistics are all-reduced once per online step (one step per
        segment) and only rank 0 writes spectra (usages stay rank-local)."""
        if run_params is None:
            run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        if not jobs:
            return
        if row_range is not None and row_segments is None:
            row_segments = [tuple(int(v) for v in row_range)]
            contiguous = True
        else:
            contiguous = False
        with self.timer("factorize"):
            kwargs = load_yaml(self.paths["nmf_run_parameters"])
            dev = _device(bool(kwargs.get("use_gpu", False)), device)
            if dev.type == "cpu" and kwargs.get("n_jobs", -1) not in (None, -1):
                torch.set_num_threads(max(1, int(kwargs["n_jobs"])))
            row_map = schedule = None
            Xd = None
            if row_segments is None:
                norm_counts = self._read_norm_counts(dev, factorize=True)
                Xd = _resident_X(norm_counts, dev) if norm_counts.X is None else None
                Xh = norm_counts.X
                cell_idx = np.arange(norm_counts.shape[0])
            else:
                from .parallel.runner import dp_layout
                from .utils.h5ad import read_X_row_segments, read_h5ad_annotations

                norm_counts = read_h5ad_annotations(self.paths["normalized_counts"])
                Xh = read_X_row_segments(self.paths["normalized_counts"], row_segments)
                row_map, schedule = dp_layout(row_segments)
                if contiguous:          # one block: the solver's own chunking
                    schedule = None
                cell_idx = np.concatenate([np.arange(a, b) for a, b in row_segments]) \
                    if row_segments else np.zeros(0, dtype=np.int64)
            X = Xd if Xd is not None else torch.from_numpy(_dense32(Xh)).to(dev)
            del Xh, Xd
            genes = norm_counts.var.index
            cells = norm_counts.obs.index[cell_idx]
            writer = comm is None or comm.rank == 0
            fault_after = int(os.environ.get("CNMF_FAULT_AFTER_REPLICATES", "0") or 0)
            written = 0
            # replicate files are encoded + hashed + written by a small thread pool (numpy
            # and zlib drop the GIL) while the next batch runs on the GPU; every file is
            # still atomic, and its sha256 is taken from the bytes in memory
            pool = cf.ThreadPoolExecutor(max_workers=4)
            pending: list = []
            manifest = self.paths["replicate_manifest"]
            gene_arr = np.asarray(genes.values).astype(str)

            def _write_batch(paths_b, W_, offs_, ks_, its_):
                if NPZ_TMP_LEVEL <= 0:
                    done = write_spectra_batch(paths_b, W_, offs_, ks_, gene_arr)
                else:
                    done = [save_arrays_npz_digest(
                        p_, {"data": W_[o_:o_ + k_], "index": np.arange(1, k_ + 1),
                             "columns": gene_arr}, level=NPZ_TMP_LEVEL)
                        for p_, o_, k_ in zip(paths_b, offs_, ks_)]
                return [{"k": int(k_), "iter": int(i_), "file": os.path.basename(p_),
                         "sha256": d_, "bytes": int(n_)}
                        for p_, k_, i_, (d_, n_) in zip(paths_b, ks_, its_, done)]

            # where the stage's time goes (bench_e2e reports it): the solves vs the wait for
            # the replicate files -- a filesystem-bound tail (900 atomic small-file writes)
            # that varies from host to host
            self.factorize_stats = {"solve_s": 0.0, "write_wait_s": 0.0}

            def _flush():
                recs = []
                t_w = time.perf_counter()
                for f in pending:
                    r_ = f.result()
                    if isinstance(r_, list):
                        recs.extend(r_)
                pending.clear()
                self.factorize_stats["write_wait_s"] += time.perf_counter() - t_w
                append_jsonl_many(manifest, recs)

            nc = run_params["n_components"].to_numpy().astype(np.int64)
            itv = run_params["iter"].to_numpy().astype(np.int64)
            sdv = run_params["nmf_seed"].to_numpy().astype(np.int64)
            jobs = sorted(jobs, key=lambda i: (int(nc[i]), i))
            solver = NMFBatchSolver(X, self._solver_options(kwargs, int(nc[jobs[0]])),
                                    comm=comm, row_map=row_map, schedule=schedule)
            # Frobenius: the whole K x n_iter grid is ONE ragged batch (one pass loop, one
            # data-side GEMM per chunk for every K) as far as device memory allows;
            # beta != 2 solves one K at a time
            for grp in self._job_batches(X, jobs, nc, dev, replicate_batch, comm,
                                         mixed=solver.beta == 2.0):
                if verbose:
                    for idx in grp:
                        print("[Worker %s]. Starting task %d." % (worker_label, idx), flush=True)
                seeds = [int(sdv[i]) for i in grp]
                ks = [int(nc[i]) for i in grp]
                t0 = time.perf_counter()
                # (writing replicates that finish early while the batch still solves was
                # measured SLOWER on the PBMC-scale grid -- factorize 350-456 vs 157-250
                # ms, profiles/r2_early_write_probe.log: the writer threads take the CPU
                # from the host enqueue -- so every file is written after its batch)
                # continuous batching when a K has more replicates than one co-resident
                # round of its usage solve holds (NMFBatchSolver.run_stream; else the
                # one-batch run): usages are only kept when they are saved
                res = solver.run_stream(seeds, ks=ks, keep_usages=save_usages)
                W = res.W.cpu().numpy()
                wall = time.perf_counter() - t0
                self.factorize_stats["solve_s"] += wall
                log.info("K=%s: %d replicates in %.3f s (%.1f replicates/s) on %s",
                         sorted(set(ks)), len(grp), wall, len(grp) / max(wall, 1e-9), dev)
                recs = []
                # fault injection (tests): only the replicates before the fault are written
                n_ok = len(grp) if not fault_after else max(0, min(len(grp), fault_after - written))
                if writer and n_ok:
                    # every replicate file of the batch not written early, in one native
                    # multi-threaded call (utils.io.write_spectra_batch), overlapped with
                    # the next batch's solve
                    rest_ = list(range(n_ok))
                    if rest_:
                        paths_b = [self.paths["iter_spectra"] % (ks[r], int(itv[grp[r]]))
                                   for r in rest_]
                        pending.append(pool.submit(
                            _write_batch, paths_b, W, [int(res.offs[r]) for r in rest_],
                            [ks[r] for r in rest_], [int(itv[grp[r]]) for r in rest_]))
                    if collect is not None:
                        collect["genes"] = gene_arr
                        for r, i in enumerate(grp[:n_ok]):
                            o = int(res.offs[r])
                            collect[(ks[r], int(itv[i]))] = W[o:o + ks[r]]
                for r, idx in enumerate(grp):
                    k, it = ks[r], int(itv[idx])
                    if writer:
                        recs.append({
                            "k": k, "iter": it, "seed": seeds[r], "worker": worker_label,
                            "err": float(res.err[r]), "n_pass": int(res.n_iter[r]),
                            "converged": bool(res.converged[r]),
                            "h_inner_iters": int(res.stats["h_inner_iters"][r]),
                            "w_inner_iters": int(res.stats["w_inner_iters"][r]),
                            "batch_size": len(grp), "batch_wall_s": wall,
                            "device": str(dev),
                            "world": 1 if comm is None else comm.world_size})
                    if save_usages:
                        us = pd.DataFrame(res.usages(r).cpu().numpy(), index=cells,
                                          columns=np.arange(1, k + 1))
                        fn = self.paths["iter_usages"] % (k, it)
                        if comm is not None and comm.world_size > 1:
                            fn = fn.replace(".df.npz", ".rank%d.df.npz" % comm.rank)
                        pending.append(pool.submit(lambda d, f: save_df_to_npz(d, f), us, fn))
                    written += 1
                    if fault_after and written >= fault_after:
                        append_jsonl_many(self.paths["replicate_log"], recs)
                        _flush()
                        pool.shutdown()
                        raise RuntimeError(
                            f"CNMF_FAULT_AFTER_REPLICATES={fault_after}: injected failure")
                append_jsonl_many(self.paths["replicate_log"], recs)
            _flush()
            pool.shutdown()

    def _job_batches(self, X: torch.Tensor, jobs, nc, dev, replicate_batch, comm, mixed):
        """Consecutive runs of the K-sorted ``jobs`` solved as one batch each: up to
        ``replicate_batch`` replicates, within ~40 % of free device memory, and (unless
        ``mixed``) of a single K.  Identical on every rank under DP."""
        N, G = X.shape
        per_row = 4 * (N + 3 * G + 2 * min(N, 5000)) + 64
        if dev.type == "cuda":
            free, _ = torch.cuda.mem_get_info(dev)
            budget = int(0.4 * free)
        else:
            budget = int(8e9)
        max_rows = max(1, budget // per_row)
        max_reps = int(replicate_batch) if replicate_batch else 1 << 30
        if comm is not None:
            max_rows = -comm.allreduce_max_int(-max_rows)
            max_reps = -comm.allreduce_max_int(-max_reps)
        out, cur, rows = [], [], 0
        for i in jobs:
            k = int(nc[i])
            if cur and (len(cur) >= max_reps or rows + k > max_rows
                        or (not mixed and int(nc[cur[-1]]) != k)):
                out.append(cur)
                cur, rows = [], 0
            cur.append(i)
            rows += k
        if cur:
            out.append(cur)
        return out

    def verify_replicates(self, components=None) -> list[dict]:
        """Check every replicate spectra file against the write manifest (sha256 recorded
        after each atomic write).  Returns one record per problem: missing file, file not
        in the manifest, or checksum mismatch (SURVEY.md §5.2 sidecar manifest)."""
        run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        latest = {}
        for rec in read_jsonl(self.paths["replicate_manifest"]):
            latest[rec["file"]] = rec
        problems = []
        for _, p in run_params.iterrows():
            k, it = int(p["n_components"]), int(p["iter"])
            if components is not None and k not in set(components):
                continue
            fn = self.paths["iter_spectra"] % (k, it)
            base = os.path.basename(fn)
            if not os.path.exists(fn):
                problems.append({"k": k, "iter": it, "problem": "missing"})
            elif base not in latest:
                problems.append({"k": k, "iter": it, "problem": "not in manifest"})
            elif _sha256(fn) != latest[base]["sha256"]:
                problems.append({"k": k, "iter": it, "problem": "checksum mismatch"})
        return problems

    # ------------------------------------------------------------------ combine
    def combine(self, components=None, skip_missing_files=False):
        if isinstance(components, (int, np.integer)):
            ks = [int(components)]
        elif components is None:
            run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
            ks = sorted(set(int(k) for k in run_params.n_components))
        else:
            ks = components
        # the K merges are independent; their zlib work runs concurrently (GIL released)
        with cf.ThreadPoolExecutor(max_workers=max(1, min(len(ks), 8))) as ex:
            list(ex.map(lambda k: self.combine_nmf(k, skip_missing_files=skip_missing_files),
                        ks))

    def combine_nmf(self, k, skip_missing_files=False, remove_individual_iterations=False):
        """Concatenate replicate spectra for one K (cnmf.py:895-920)."""
        run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        print("Combining factorizations for k=%d." % k)
        sub = run_params[run_params.n_components == k].sort_values("iter")
        present = []
        for _, p in sub.iterrows():
            fn = self.paths["iter_spectra"] % (int(p["n_components"]), int(p["iter"]))
            if not os.path.exists(fn):
                if not skip_missing_files:
                    print("Missing file: %s, run with skip_missing=True to override" % fn)
                    raise FileNotFoundError(errno.ENOENT, os.strerror(errno.ENOENT), fn)
                print("Missing file: %s. Skipping." % fn)
                continue
            present.append((int(p["iter"]), fn))
        native = read_spectra_batch([fn for _, fn in present]) if present else None
        if native is not None:     # stored npz parsed on native threads (csrc/io/npzio.cpp)
            data, kk, cols = native
            if any(int(x) != int(k) for x in kk):
                raise ValueError(f"k={k}: a replicate file holds a different number of "
                                 "components")
            index = ["iter%d_topic%d" % (it, t + 1) for it, _ in present for t in range(k)]
            combined = pd.DataFrame(data, index=index, columns=cols)
            save_df_to_npz(combined, self.paths["merged_spectra"] % k, level=NPZ_TMP_LEVEL)
            if remove_individual_iterations:
                for _, p in sub.iterrows():
                    fn = self.paths["iter_spectra"] % (int(p["n_components"]), int(p["iter"]))
                    if os.path.exists(fn):
                        os.remove(fn)
            return combined
        with cf.ThreadPoolExecutor(max_workers=8) as ex:   # zlib inflate drops the GIL
            loaded = list(ex.map(lambda t: _load_npz_arrays(t[1]), present))
        if loaded:
            # one concatenated array instead of one DataFrame per replicate (pd.concat of
            # 100 frames with 2k string columns was the cost of this stage); every
            # replicate must carry the same gene columns
            cols = loaded[0][2]
            for (_, fn), (_, _, c) in zip(present, loaded):
                if c.shape != cols.shape or not np.array_equal(c, cols):
                    raise ValueError(f"{fn}: gene columns differ from the other replicates")
            index = ["iter%d_topic%d" % (it, t + 1) for it, _ in present for t in range(k)]
            combined = pd.DataFrame(np.concatenate([d for d, _, _ in loaded], axis=0),
                                    index=index, columns=cols)
            save_df_to_npz(combined, self.paths["merged_spectra"] % k, level=NPZ_TMP_LEVEL)
            if remove_individual_iterations:
                for _, p in sub.iterrows():
                    fn = self.paths["iter_spectra"] % (int(p["n_components"]), int(p["iter"]))
                    if os.path.exists(fn):
                        os.remove(fn)
            return combined
        print("No spectra found for k=%d" % k)
        return []

    # ------------------------------------------------------------------ refits
    def _refit_kwargs(self):
        """The run parameters YAML, parsed once per file version (k-selection re-read it
        twice per K: ~30 ms of PyYAML per run)."""
        fn = self.paths["nmf_run_parameters"]
        st = os.stat(fn)
        key = (fn, st.st_mtime_ns, st.st_size)
        cache = getattr(self, "_yaml_cache", None)
        if cache is None or cache[0] != key:
            cache = (key, load_yaml(fn))
            self._yaml_cache = cache
        return dict(cache[1])

    def refit_usage(self, X, spectra, usage=None, device=None):
        """Refit usages with spectra fixed (cnmf.py:923-976): online MU, h_tol 0.05."""
        kw = self._refit_kwargs()
        dev = _device(bool(kw.get("use_gpu", False)), device)
        return fit_H_online(X, spectra, H_init=usage, chunk_size=kw["online_chunk_size"],
                            chunk_max_iter=kw["online_chunk_max_iter"], h_tol=0.05,
                            l1_reg_H=kw.get("l1_ratio_H", 0.0), l2_reg_H=0.0, epsilon=1e-16,
                            device=dev)

    def refit_spectra(self, X, usage, device=None, comm=None):
        """Refit spectra with usages fixed (cnmf.py:979-994).  With a multi-rank ``comm``
        the genes are sharded over the ranks in whole refit chunks (tensor/gene-axis
        parallelism) and the K x G blocks are all-gathered."""
        kw = self._refit_kwargs()
        dev = _device(bool(kw.get("use_gpu", False)), device)
        u = usage.values if isinstance(usage, pd.DataFrame) else np.asarray(usage)
        args = dict(chunk_size=kw["online_chunk_size"], chunk_max_iter=kw["online_chunk_max_iter"],
                    h_tol=0.05, l1_reg=kw.get("l1_ratio_H", 0.0), device=dev)
        if comm is None or comm.world_size == 1:
            return fit_spectra_online(X, u, **args)
        g0, g1 = gene_blocks(X.shape[1], kw["online_chunk_size"], comm.world_size)[comm.rank]
        part = fit_spectra_online(col_block(X, g0, g1), u, col_offset=g0, **args) if g1 > g0 \
            else np.zeros((u.shape[1], 0), dtype=np.float32)
        return np.concatenate(comm.all_gather_object(part), axis=1)

    # ------------------------------------------------------------------ consensus
    def consensus(self, k, density_threshold=0.5, local_neighborhood_size=0.30,
                  show_clustering=True, build_ref=True, skip_density_and_return_after_stats=False,
                  close_clustergram_fig=False, refit_usage=True, normalize_tpm_spectra=False,
                  norm_counts=None, kmeans_backend="auto", device=None, comm=None,
                  wait_figures=True):
        """Consensus spectra/usages for one K (cnmf.py:997-1256).  With a multi-rank
        ``comm`` the two all-gene passes -- the TPM spectra refit and the OLS gene scores
        over G_all -- are sharded over the ranks by gene blocks (the clustering is
        replicated); rank 0 writes the artifacts.  ``wait_figures=False`` (closed figures
        only): return before the clustergram PNG is written; it finishes while the caller
        goes on (utils.plotting.flush_figures, which the CLI calls before exiting)."""
        with self.timer(f"consensus_k{k}"):
            return self._consensus(k, density_threshold, local_neighborhood_size, show_clustering,
                                   build_ref, skip_density_and_return_after_stats,
                                   close_clustergram_fig, refit_usage, normalize_tpm_spectra,
                                   norm_counts, kmeans_backend, device, comm, wait_figures)

    def _consensus(self, k, density_threshold, local_neighborhood_size, show_clustering,
                   build_ref, skip_stats, close_fig, refit_usage, normalize_tpm_spectra,
                   norm_counts, kmeans_backend, device, comm=None, wait_figures=True):
        tp = comm is not None and comm.world_size > 1
        writer = not tp or comm.rank == 0
        # a closed clustergram is drawn by a child process that imports matplotlib while
        # this stage computes (utils.plotting.PlotWorker)
        plot_worker = None
        if show_clustering and close_fig and writer and not skip_stats and \
                "matplotlib.pyplot" not in sys.modules:
            from .utils.plotting import PlotWorker

            plot_worker = PlotWorker()
        kw = self._refit_kwargs()
        dev = _device(bool(kw.get("use_gpu", False)), device)
        merged = load_df_from_npz(self.paths["merged_spectra"] % k)
        if norm_counts is None:
            norm_counts = self._read_norm_counts(dev)
        dt_str = "2" if skip_stats else str(density_threshold)
        dt_repl = dt_str.replace(".", "_")
        n_neighbors = int(local_neighborhood_size * merged.shape[0] / k)

        # float32 spectra cross to the device as float32 (half the bytes) and widen there
        mv = np.ascontiguousarray(merged.values)
        S = torch.from_numpy(mv).to(dev).to(torch.float64) if mv.dtype == np.float32 else \
            torch.as_tensor(mv, dtype=torch.float64, device=dev)
        L2 = l2_normalize_rows(S)
        names = merged.index
        topics_dist = None
        density_filter = None
        local_dens = None
        if not skip_stats:
            cache = self.paths["local_density_cache"] % k
            local_dens = self._load_density_cache(cache, n_neighbors, names)
            if local_dens is None:
                topics_dist = pairwise_distances(L2)
                dens = local_density(topics_dist, n_neighbors).cpu().numpy()
                local_dens = pd.DataFrame(dens, columns=["local_density"], index=names)
                if writer:
                    save_df_to_npz(local_dens, cache)
                    write_text_atomic(cache + ".meta.json", json.dumps(
                        {"n_neighbors": n_neighbors, "n_spectra": int(len(names))}))
            density_filter = (local_dens.iloc[:, 0] < density_threshold).values
            keep = torch.as_tensor(np.flatnonzero(density_filter), device=dev)
            L2 = L2.index_select(0, keep)
            names = names[density_filter]
            if L2.shape[0] == 0:
                raise RuntimeError("Zero components remain after density filtering. Consider "
                                   "increasing density threshold")
        labels = kmeans(L2, k, n_init=10, random_state=1, backend=kmeans_backend) + 1
        label_series = pd.Series(labels, index=names)
        if plot_worker is not None:
            # the clustergram needs only the clustering: hand it to the figure child now,
            # so it renders while the refits / OLS / writes below run
            if topics_dist is None:
                topics_dist = pairwise_distances(L2)
            else:
                keep_t = torch.as_tensor(np.flatnonzero(density_filter), device=topics_dist.device)
                topics_dist = topics_dist.index_select(0, keep_t).index_select(1, keep_t)
            plot_worker.submit(
                "clustergram", self.paths["clustering_plot"] % (k, dt_repl),
                dist=topics_dist.cpu().numpy(), labels=label_series.values,
                names=np.asarray(label_series.index).astype(str),
                local_density=(local_dens.values.reshape(-1) if local_dens is not None
                               else np.zeros(0)),
                density_filter=(density_filter if density_filter is not None
                                else np.zeros(0, dtype=bool)),
                density_threshold=np.float64(density_threshold))
        median_np = cluster_medians(L2, labels, sorted(set(labels))).cpu().numpy()
        median_spectra = pd.DataFrame(median_np, index=sorted(set(labels)), columns=merged.columns)

        ncX = _resident_X(norm_counts, dev)
        # the usage refit's cooperative solves spin on their own workgroups' progress,
        # so two of them must not share the GPU: serialised across the k-selection
        # threads (everything else of a K -- npz read, k-means, medians -- overlaps)
        with _COOP_LOCK:
            rf_usages = self.refit_usage(ncX, median_spectra, device=dev)
        rf_usages = pd.DataFrame(rf_usages, index=norm_counts.obs.index, columns=median_spectra.index)

        if skip_stats:
            d = pairwise_distances(L2)
            sil = silhouette(d, labels)
            err = self._prediction_error(ncX, rf_usages.values, median_spectra.values, dev)
            return pd.DataFrame([k, density_threshold, sil, err],
                                index=["k", "local_density_threshold", "silhouette",
                                       "prediction_error"], columns=["stats"])

        norm_usages = rf_usages.div(rf_usages.sum(axis=1), axis=0)
        reorder = norm_usages.sum(axis=0).sort_values(ascending=False)
        rf_usages = rf_usages.loc[:, reorder.index]
        norm_usages = norm_usages.loc[:, reorder.index]
        median_spectra = median_spectra.loc[reorder.index, :]
        new_cols = np.arange(1, rf_usages.shape[1] + 1)
        rf_usages.columns = new_cols
        norm_usages.columns = new_cols
        median_spectra.index = new_cols

        tpm = resident.recall(self.paths["tpm"], "adata")
        if tpm is None:
            tpm = read_h5ad(self.paths["tpm"])
        tpm_stats = load_df_from_npz(self.paths["tpm_stats"])
        # sparse TPM on the GPU: uploaded once as CSR; the spectra refit, the OLS and the
        # scaled-HVG usage refit below are CSR kernel passes over it (ops.sparse)
        dT = _device_csr_cached(tpm, dev)
        tpmX = dT if dT is not None else tpm.X
        spectra_tpm = self.refit_spectra(tpmX, norm_usages.astype(tpm.X.dtype), device=dev,
                                         comm=comm if tp else None)
        spectra_tpm = pd.DataFrame(spectra_tpm, index=new_cols, columns=tpm.var.index)
        if normalize_tpm_spectra:
            spectra_tpm = spectra_tpm.div(spectra_tpm.sum(axis=1), axis=0) * 1e6

        if tp:   # gene-sharded OLS: each rank z-scores and solves its gene block
            g0, g1 = gene_blocks(tpm.shape[1], self._refit_kwargs()["online_chunk_size"],
                                 comm.world_size)[comm.rank]
            part = efficient_ols_all_cols(rf_usages.values, col_block(tpmX, g0, g1),
                                          normalize_y=True, device=dev) if g1 > g0 else \
                np.zeros((rf_usages.shape[1], 0))
            usage_coef = np.concatenate(comm.all_gather_object(part), axis=1)
        else:
            usage_coef = efficient_ols_all_cols(rf_usages.values, tpmX, normalize_y=True,
                                                device=dev)
        usage_coef = pd.DataFrame(usage_coef, index=new_cols, columns=tpm.var.index)

        if refit_usage:
            with open(self.paths["nmf_genes_list"]) as fh:
                hvgs = fh.read().split("\n")
            if dT is not None:
                # scale(tpm[:, hvgs], zero_center=False) as a lazy view of the resident CSR
                pos = tpm.var.index.get_indexer(hvgs)
                if (pos < 0).any():
                    raise KeyError(f"HVGs missing from the TPM matrix: {list(np.array(hvgs)[pos < 0][:5])}")
                cmap = np.full(tpm.shape[1], -1, np.int32)
                cmap[pos] = np.arange(len(hvgs), dtype=np.int32)
                _, var = sops.mean_var(dT, ddof=1, col_map=cmap, n_out=len(hvgs))
                std = torch.sqrt(var)
                std[std == 0] = 1.0
                norm_X = dT.view(col_map=cmap, col_div=std, n_out=len(hvgs))
                norm_dtype = tpm.X.dtype
            else:
                norm_tpm = tpm[:, hvgs]
                if sp.issparse(norm_tpm.X):
                    norm_tpm = pp_scale(norm_tpm, zero_center=False)
                else:
                    norm_tpm.X = norm_tpm.X / norm_tpm.X.std(axis=0, ddof=1)
                norm_X, norm_dtype = norm_tpm.X, norm_tpm.X.dtype
            spectra_tpm_rf = spectra_tpm.loc[:, hvgs]
            spectra_tpm_rf = spectra_tpm_rf.div(tpm_stats.loc[hvgs, "__std"], axis=1)
            rf = self.refit_usage(norm_X, spectra_tpm_rf.astype(norm_dtype), device=dev)
            rf_usages = pd.DataFrame(rf, index=norm_counts.obs.index, columns=spectra_tpm_rf.index)
        del dT, tpmX

        if not writer:
            return None
        p = self.paths
        # the eight artifacts are independent atomic files: written by a few threads
        # (zlib and the native TSV writer drop the GIL; ~1 s serial at 500k cells)
        outs = [(save_df_to_npz, median_spectra, "consensus_spectra"),
                (save_df_to_npz, rf_usages, "consensus_usages"),
                (save_df_to_text, median_spectra, "consensus_spectra__txt"),
                (save_df_to_text, rf_usages, "consensus_usages__txt"),
                (save_df_to_npz, spectra_tpm, "gene_spectra_tpm"),
                (save_df_to_text, spectra_tpm, "gene_spectra_tpm__txt"),
                (save_df_to_npz, usage_coef, "gene_spectra_score"),
                (save_df_to_text, usage_coef, "gene_spectra_score__txt")]
        with cf.ThreadPoolExecutor(max_workers=4) as ex:
            for f in [ex.submit(fn, df, p[key] % (k, dt_repl)) for fn, df, key in outs]:
                f.result()

        if show_clustering and plot_worker is None:
            from .utils.plotting import clustergram

            if topics_dist is None:
                topics_dist = pairwise_distances(L2)
            else:
                keep = torch.as_tensor(np.flatnonzero(density_filter), device=topics_dist.device)
                topics_dist = topics_dist.index_select(0, keep).index_select(1, keep)
            clustergram(topics_dist.cpu().numpy(), label_series, local_dens, density_filter,
                        density_threshold, p["clustering_plot"] % (k, dt_repl), close=close_fig)
        if build_ref:
            # the reference re-reads the TSV it just wrote (cnmf.py:1273); float64 text is
            # an exact round trip, so the in-memory frame gives the same reference
            mem = spectra_tpm if (spectra_tpm.dtypes == np.float64).all() else None
            self.build_reference(k, density_threshold, _spectra_tpm=mem)
        if plot_worker is not None:
            plot_worker.wait(defer=not wait_figures)

    def _load_density_cache(self, cache: str, n_neighbors: int, names):
        """Density cache keyed on K AND the neighbourhood (SURVEY.md §5.2 fix): a cache
        written with a different n_neighbors or spectra set is recomputed."""
        if not os.path.isfile(cache):
            return None
        meta_fn = cache + ".meta.json"
        if os.path.isfile(meta_fn):
            with open(meta_fn) as fh:
                meta = json.load(fh)
            if meta.get("n_neighbors") != n_neighbors or meta.get("n_spectra") != len(names):
                return None
        df = load_df_from_npz(cache)
        if len(df) != len(names):
            return None
        return df

    @staticmethod
    def _prediction_error(X, usages: np.ndarray, spectra: np.ndarray, dev) -> float:
        """||X - U S||_F^2 via the trace identity, streamed (never materialises U S).  A
        device-resident X (dense tensor or DeviceCSR, see _resident_X) is used in place."""
        U = torch.as_tensor(usages, dtype=torch.float64, device=dev)
        S = torch.as_tensor(spectra, dtype=torch.float64, device=dev)
        quad = float((ops.small_gram(U) * ops.small_gram(S, rows_are_points=False)).sum())
        if isinstance(X, sops.DeviceCSR) and not X.xf:
            d = X.data.to(torch.float64)
            UtX = sops.tspmm(X, U).t().to(torch.float64)              # (K, G)
            return float((d * d).sum()) - 2.0 * float((UtX * S).sum()) + quad
        if isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32 \
                and U.shape[1] <= 128:
            # one fused pass over the resident X (H8 kernel): <X, U S> and ||X||^2
            cross, x_sq = sops_predict(X, U, S)
            return x_sq - 2.0 * cross + quad
        if isinstance(X, torch.Tensor):
            # ||X||^2 is the same for every K of a k-selection: computed once per tensor
            x_sq = _XSQ.get(X)
            cross = torch.zeros((), dtype=torch.float64, device=dev)
            xs = None if x_sq is not None else torch.zeros((), dtype=torch.float64, device=dev)
            for a in range(0, X.shape[0], 16384):
                xb = X[a:a + 16384].to(device=dev, dtype=torch.float64)
                if xs is not None:
                    xs += (xb * xb).sum()
                cross += ((U[a:a + 16384].t() @ xb) * S).sum()
            if xs is not None:
                x_sq = float(xs)
                _XSQ[X] = x_sq
            return x_sq - 2.0 * float(cross) + quad
        n = X.shape[0]
        x_sq = 0.0
        cross = 0.0
        for a in range(0, n, 16384):
            b = min(n, a + 16384)
            blk = X[a:b]
            blk = blk.toarray() if sp.issparse(blk) else np.asarray(blk)
            xb = torch.as_tensor(blk, dtype=torch.float64, device=dev)
            x_sq += float((xb * xb).sum())
            cross += float(((U[a:b].t() @ xb) * S).sum())
        quad = float((ops.small_gram(U) * ops.small_gram(S, rows_are_points=False)).sum())
        return x_sq - 2.0 * cross + quad

    # ------------------------------------------------------------------ reference / k-sel
    def build_reference(self, k, density_threshold=0.5, target_sum=1e6, _spectra_tpm=None):
        """starCAT reference spectra (cnmf.py:1259-1290)."""
        dt = _dt_str(density_threshold)
        if _spectra_tpm is not None:
            spectra_tpm = _spectra_tpm.copy()
            spectra_tpm.columns = spectra_tpm.columns.astype(str)
        else:
            # the reference's read (cnmf.py:1273), whole-file and memory-mapped: the same
            # C parser and values, without the per-chunk type inference (0.15 -> 0.09 s
            # for 8000 genes)
            spectra_tpm = pd.read_csv(self.paths["gene_spectra_tpm__txt"] % (k, dt),
                                      index_col=0, sep="\t", low_memory=False,
                                      memory_map=True)
        with open(self.paths["nmf_genes_list"]) as fh:
            hvgs = fh.read().split("\n")
        tpm_stats = load_df_from_npz(self.paths["tpm_stats"])
        tpm_stats.index = spectra_tpm.columns
        renorm = spectra_tpm.div(spectra_tpm.sum(axis=1), axis=0) * target_sum
        varnorm = renorm.div(tpm_stats["__std"])
        ref = varnorm[hvgs].copy()
        ref.index = "GEP" + ref.index.astype("str")
        save_df_to_npz(ref, self.paths["starcat_spectra"] % (k, dt))
        save_df_to_text(ref, self.paths["starcat_spectra__txt"] % (k, dt))

    def k_selection_plot(self, close_fig=False, kmeans_backend="auto", comm=None,
                         device=None, wait_figures=True):
        """Stability (silhouette) and error per K (cnmf.py:1293-1332).

        With ``comm`` (one rank per GPU) the Ks are dealt round-robin over the ranks, each
        rank runs its Ks' stats on its own device, and rank 0 gathers the rows (Python
        objects, a few floats per K) and writes the npz and the plot."""
        run_params = load_df_from_npz(self.paths["nmf_replicate_parameters"])
        rank, world = (0, 1) if comm is None else (comm.rank, comm.world_size)
        plot_worker = None
        if close_fig and rank == 0 and "matplotlib.pyplot" not in sys.modules:
            from .utils.plotting import PlotWorker

            plot_worker = PlotWorker()   # imports matplotlib while the stats compute
        dev = _device(bool(self._refit_kwargs().get("use_gpu", False)), device)
        norm_counts = self._read_norm_counts(dev)
        ks = sorted(set(int(x) for x in run_params.n_components))
        mine = ks[rank::world]

        def stats_of(k):
            return self.consensus(k, skip_density_and_return_after_stats=True,
                                  show_clustering=False, close_clustergram_fig=True,
                                  norm_counts=norm_counts, kmeans_backend=kmeans_backend,
                                  device=device).stats

        rows = {}
        if dev.type == "cuda" and len(mine) > 1:
            # the Ks are independent and each is a chain of small kernels and host reads:
            # run them on a few threads with a HIP stream each, so one K's host syncs,
            # npz reads and k-means checks overlap the others' GPU work.  X is uploaded
            # once, before the threads start
            _resident_X(norm_counts, dev)
            torch.cuda.synchronize(dev)

            local = threading.local()

            def on_stream(k):
                s = getattr(local, "stream", None)
                if s is None:
                    s = local.stream = torch.cuda.Stream(dev)
                with torch.cuda.stream(s):
                    out = stats_of(k)
                s.synchronize()
                return out

            with cf.ThreadPoolExecutor(max_workers=min(_KSEL_THREADS, len(mine))) as ex:
                for k, st in zip(mine, ex.map(on_stream, mine)):
                    rows[k] = st
        else:
            for k in mine:
                rows[k] = stats_of(k)
        if world > 1:
            for part in comm.all_gather_object(rows):
                rows.update(part)
            if rank != 0:
                return None
        stats = pd.DataFrame([rows[k] for k in ks]).reset_index(drop=True)
        save_df_to_npz(stats, self.paths["k_selection_stats"])
        if plot_worker is not None:
            plot_worker.submit("k_selection", self.paths["k_selection_plot"],
                               k=stats["k"].to_numpy(dtype=np.float64),
                               silhouette=stats["silhouette"].to_numpy(dtype=np.float64),
                               prediction_error=stats["prediction_error"].to_numpy(
                                   dtype=np.float64))
            plot_worker.wait(defer=not wait_figures)
        else:
            from .utils.plotting import k_selection

            k_selection(stats, self.paths["k_selection_plot"], close=close_fig)
        return stats

    def load_results(self, K, density_threshold, n_top_genes=100, norm_usage=True):
        """(usage, spectra_scores, spectra_tpm, top_genes) (cnmf.py:1335-1384)."""
        dt = _dt_str(density_threshold)
        spectra_scores = pd.read_csv(self.paths["gene_spectra_score__txt"] % (K, dt), sep="\t",
                                     index_col=0).T
        spectra_tpm = pd.read_csv(self.paths["gene_spectra_tpm__txt"] % (K, dt), sep="\t",
                                  index_col=0).T
        usage = pd.read_csv(self.paths["consensus_usages__txt"] % (K, dt), sep="\t", index_col=0)
        if norm_usage:
            usage = usage.div(usage.sum(axis=1), axis=0)
        try:
            usage.columns = [int(x) for x in usage.columns]
        except ValueError:
            print("Usage matrix columns include non integer values")
        top_genes = []
        for gep in spectra_scores.columns:
            top_genes.append(list(spectra_scores.sort_values(by=gep, ascending=False)
                                  .index[:n_top_genes]))
        top_genes = pd.DataFrame(top_genes, index=spectra_scores.columns).T
        return usage, spectra_scores, spectra_tpm, top_genes

"""``Preprocess``: QC filtering, normalisation, HVG selection and Harmony batch
correction of expression data before cNMF (C30-C38; preprocess.py:41-439).

Same methods, arguments and outputs as the reference.  scanpy/harmonypy calls are
replaced by :mod:`.models.pp` and :mod:`.models.harmony` (device-resident); the MOE
ridge correction of the expression matrix runs as batched GEMMs on the GPU when one is
available (``device`` argument / ``CNMF_DEVICE``).  Two plotting bugs of the reference
are fixed: the n_counts histogram marks ``min_counts_per_cell``
and the mito histogram title is set with ``set_title``.
"""
from __future__ import annotations

import os
from collections.abc import Collection

import numpy as np
import pandas as pd
import scipy.sparse as sp
import torch

from .models import pp
from .models.harmony import moe_correct_ridge, run_harmony
from .utils.anndata_lite import AnnData, to_lite
from .utils.h5ad import write_h5ad
from .utils.io import write_text_atomic
from .utils.transfer import to_host


_WRITER = None


def _writer():
    """One background thread for output files written while the device keeps working."""
    global _WRITER
    if _WRITER is None:
        import concurrent.futures as cf
        _WRITER = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="cnmf-write")
    return _WRITER


def _default_device():
    env = os.environ.get("CNMF_DEVICE")
    if env:
        return torch.device(env)
    from .utils.gpu import visible

    return torch.device("cuda") if visible() else torch.device("cpu")


def stdscale_quantile_celing(_adata, max_value=None, quantile_thresh=None):
    """Scale genes to unit variance (no centring), cap at ``max_value`` and at the
    global ``quantile_thresh`` quantile (preprocess.py:21-29).  The quantile is taken
    over ALL entries (zeros included) like the reference, but without densifying a
    sparse matrix: the zeros' share of the order statistics is accounted analytically."""
    ad = pp.scale(_adata, zero_center=False, max_value=max_value)
    if quantile_thresh is not None:
        X = ad.X
        if sp.issparse(X):
            n_total = X.shape[0] * X.shape[1]
            n_zero = n_total - X.data.size
            # np.quantile (linear) over the virtual full vector [zeros..., data...]
            # (scaled counts are >= 0); only the two order statistics needed are selected
            # (O(nnz) partition, not a sort of all stored values)
            pos = quantile_thresh * (n_total - 1)
            lo, hi = int(np.floor(pos)), int(np.ceil(pos))
            if X.data.size and X.data.min() < 0:
                full = np.concatenate([np.zeros(n_zero, X.data.dtype), X.data])
                thr = float(np.quantile(full, quantile_thresh))
            else:
                want = sorted({i - n_zero for i in (lo, hi) if i >= n_zero})
                part = np.partition(X.data, want) if want else None

                def at(i):
                    return 0.0 if i < n_zero else float(part[i - n_zero])

                thr = at(lo) + (at(hi) - at(lo)) * (pos - lo)
            np.minimum(X.data, X.data.dtype.type(thr), out=X.data)
        else:
            thr = np.quantile(X.reshape(-1), quantile_thresh)
            X[X > thr] = thr
        ad.X = X
    return ad


def make_count_hist(adata, num_cells=1000):
    from .utils.plotting import count_hist

    return count_hist(adata.X, num_cells)


class Preprocess:
    def __init__(self, random_seed=None):
        np.random.seed(random_seed)
        self.random_seed = random_seed

    def filter_adata(self, _adata, filter_mito_thresh=None, min_cells_per_gene=10,
                     min_counts_per_cell=500, filter_mito_genes=False, filter_dot_genes=True,
                     makeplots=True):
        """QC filters (preprocess.py:60-132)."""
        ad = to_lite(_adata)
        if min_cells_per_gene is not None:
            pp.filter_genes(ad, min_cells=min_cells_per_gene)
        ad.obs["n_counts"] = np.asarray(ad.X.sum(axis=1)).squeeze()
        if makeplots:
            from .utils.plotting import _plt

            plt = _plt()
            fig, ax = plt.subplots()
            ax.hist(np.log10(np.maximum(ad.obs["n_counts"].values, 1e-12)), bins=100)
            ax.set_title("log10 n_counts")
            ylim = ax.get_ylim()
            if min_counts_per_cell:
                ax.vlines(x=np.log10(min_counts_per_cell), ymin=ylim[0], ymax=ylim[1])
            ax.set_ylim(ylim)
        if min_counts_per_cell is not None:
            pp.filter_cells(ad, min_counts=min_counts_per_cell)
        mt_genes = [x for x in ad.var.index if "MT-" in x]
        if filter_mito_thresh is not None:
            num_mito = np.asarray(ad[:, mt_genes].X.sum(axis=1)).squeeze()
            pct = num_mito / ad.obs["n_counts"].values
            ad.obs["pct_mito"] = pct
            if makeplots:
                from .utils.plotting import _plt

                plt = _plt()
                fig, ax = plt.subplots()
                ax.hist(ad.obs["pct_mito"], bins=100)
                ax.set_title("pct_mito")
            ad = ad[ad.obs["pct_mito"].values < filter_mito_thresh, :]
        tofilter = []
        if filter_dot_genes:
            tofilter = [x for x in ad.var.index if "." in x]
        if filter_mito_genes:
            tofilter = tofilter + mt_genes
        keep = ~ad.var.index.isin(tofilter)
        return ad[:, keep]

    def preprocess_for_cnmf(self, _adata, feature_type_col=None,
                            adt_feature_name="Antibody Capture", harmony_vars=None,
                            n_top_rna_genes=2000, librarysize_targetsum=1e4,
                            max_scaled_thresh=None, quantile_thresh=.9999, makeplots=True,
                            theta=1, save_output_base=None, max_iter_harmony=20, device=None):
        """HVG-filtered, normalised, optionally Harmony-corrected input for cNMF plus a
        TP10K matrix (RNA [+ ADT]) for the tpm input (preprocess.py:135-247)."""
        if (not isinstance(_adata, Collection) or _is_anndata(_adata)) and feature_type_col is not None:
            ad = to_lite(_adata)
            is_adt = (ad.var[feature_type_col] == adt_feature_name).values
            adata_ADT = ad[:, is_adt]
            adata_RNA = ad[:, ~is_adt]
        elif not isinstance(_adata, Collection) or _is_anndata(_adata):
            adata_RNA = to_lite(_adata)
            adata_RNA.var_names_make_unique()
            adata_RNA.var["features_renamed"] = adata_RNA.var.index
            adata_ADT = None
        elif len(_adata) == 2:
            adata_RNA, adata_ADT = to_lite(_adata[0]), to_lite(_adata[1])
            if adata_ADT.shape[0] != adata_RNA.shape[0]:
                raise Exception("ADT and RNA AnnDatas don't have the same number of cells")
            if np.sum(adata_ADT.obs.index != adata_RNA.obs.index) > 0:
                raise Exception("Inconsistency of the index for the ADT and RNA AnnDatas")
        else:
            raise Exception("data should either be an AnnData object or a list of 2 AnnData objects")

        dev = torch.device(device) if device is not None else _default_device()
        dX = _device_counts(adata_RNA, dev) if harmony_vars is not None else None
        if dX is not None:
            # TP10K from the resident counts: one row-sum + one scaling pass on the device
            from .ops import sparse as sops

            rs = librarysize_targetsum / _nonzero(sops.row_sums(dX))
            f64 = adata_RNA.X.dtype == np.float64       # normalize_total keeps float64
            data = sops.transform(dX, row_scale=rs, round_mid=not f64,
                                  out_dtype=torch.float64 if f64 else torch.float32)
            data = to_host(data)
            X0 = adata_RNA.X
            tp10k = AnnData(X=sp.csr_matrix((data, X0.indices, X0.indptr), shape=X0.shape),
                            obs=adata_RNA.obs, var=adata_RNA.var,
                            obsm=dict(adata_RNA.obsm), varm=dict(adata_RNA.varm),
                            uns=dict(adata_RNA.uns))
        else:
            tp10k = pp.normalize_total(adata_RNA, target_sum=librarysize_targetsum, copy=True)
        # without ADT the TP10K file is final here: it is written on a background thread
        # (the native writer drops the GIL) while HVG / PCA / Harmony run on the device --
        # ~5 GB of CSR at 500k cells, 0.6 s of the config-5 stage (profiles/r5i_*)
        tp_write = None
        if save_output_base is not None and adata_ADT is None:
            tp_write = _writer().submit(write_h5ad, save_output_base + ".TP10K.h5ad", tp10k)
        try:
            adata_RNA, hvgs = self.normalize_batchcorrect(
                adata_RNA, harmony_vars=harmony_vars, n_top_genes=n_top_rna_genes,
                librarysize_targetsum=librarysize_targetsum, max_scaled_thresh=max_scaled_thresh,
                quantile_thresh=quantile_thresh, theta=theta, makeplots=makeplots,
                max_iter_harmony=max_iter_harmony, device=dev, _device_csr=dX)
        except BaseException:
            if tp_write is not None:
                tp_write.exception()    # no write left running behind the error
            raise
        del dX

        if adata_ADT is not None:
            adata_ADT = adata_ADT[adata_RNA.obs.index, :]
            adata_ADT = pp.normalize_total(adata_ADT, target_sum=librarysize_targetsum)
            merge_var = pd.concat([tp10k.var, adata_ADT.var], axis=0)
            Xr = tp10k[adata_RNA.obs.index, :].X
            X = sp.hstack((sp.csr_matrix(Xr), sp.csr_matrix(adata_ADT.X))).tocsr()
            tp10k = AnnData(X=X, obs=tp10k[adata_RNA.obs.index, :].obs, var=merge_var)

        if save_output_base is not None:
            write_h5ad(save_output_base + ".Corrected.HVG.Varnorm.h5ad", adata_RNA)
            if tp_write is None:
                write_h5ad(save_output_base + ".TP10K.h5ad", tp10k)
            else:
                tp_write.result()
            write_text_atomic(save_output_base + ".Corrected.HVGs.txt", "\n".join(hvgs))
        return adata_RNA, tp10k, hvgs

    def normalize_batchcorrect(self, _adata, normalize_librarysize=False, harmony_vars=None,
                               n_top_genes=None, librarysize_targetsum=1e4,
                               max_scaled_thresh=None, quantile_thresh=.9999, theta=1,
                               makeplots=True, max_iter_harmony=20, device=None,
                               _device_csr=None):
        """Seurat-v3 HVGs, scaling + quantile ceiling, optional Harmony (preprocess.py:250-338).

        On a GPU with sparse counts and ``harmony_vars``, the counts are uploaded once and
        every step runs on the device (:meth:`_harmony_device`)."""
        ad = to_lite(_adata)
        dev = torch.device(device) if device is not None else _default_device()
        dX = _device_csr
        if dX is None and harmony_vars is not None:
            dX = _device_counts(ad, dev)
        if n_top_genes is not None:
            pp.highly_variable_genes(ad, flavor="seurat_v3", n_top_genes=n_top_genes,
                                     device_csr=dX)
        elif "highly_variable" not in ad.var.columns:
            raise Exception("If a numeric value for n_top_genes is not provided, you must include "
                            "a highly_variable column in _adata")
        hv = ad.var["highly_variable"].values.astype(bool)
        if harmony_vars is not None and dX is not None:
            ad = self._harmony_device(ad, dX, hv, normalize_librarysize, harmony_vars,
                                      librarysize_targetsum, max_scaled_thresh, quantile_thresh,
                                      theta, makeplots, max_iter_harmony)
        elif harmony_vars is not None:
            anorm = pp.normalize_total(ad, target_sum=librarysize_targetsum, copy=True)
            anorm = anorm[:, hv]
            anorm = stdscale_quantile_celing(anorm, max_value=max_scaled_thresh,
                                             quantile_thresh=quantile_thresh)
            sub = ad[:, hv]
            sub = stdscale_quantile_celing(sub, max_value=max_scaled_thresh,
                                           quantile_thresh=quantile_thresh)
            if makeplots:
                make_count_hist(anorm, num_cells=1000)
            pp.pca(anorm, use_highly_variable=False, zero_center=True, device=dev)
            sub.obsm["X_pca"] = anorm.obsm["X_pca"]
            src = sub if not normalize_librarysize else anorm
            Xd = src.X.toarray() if sp.issparse(src.X) else np.asarray(src.X)
            sub.X, sub.obsm["X_pca_harmony"] = self.harmony_correct_X(
                Xd, src.obs, src.obsm["X_pca"], harmony_vars, max_iter_harmony=max_iter_harmony,
                theta=theta, device=dev)
            ad = sub
        else:
            if normalize_librarysize:
                ad = pp.normalize_total(ad, target_sum=librarysize_targetsum)
            ad = ad[:, hv]
            ad = stdscale_quantile_celing(ad, max_value=max_scaled_thresh,
                                          quantile_thresh=quantile_thresh)
            if makeplots:
                make_count_hist(ad, num_cells=1000)
        hvgs = list(ad.var.index)
        return ad, hvgs

    def _harmony_device(self, ad, A, hv, normalize_librarysize, harmony_vars, target_sum,
                        max_scaled_thresh, quantile_thresh, theta, makeplots, max_iter_harmony):
        """The harmony branch of normalize_batchcorrect (preprocess.py:300-324) with the
        counts resident on the GPU as CSR (ops.sparse): normalize_total, the HVG subset,
        scale(zero_center=False) with both ceilings and the densification are fused
        into column-statistics / densify kernel passes; PCA, Harmony and the MOE ridge
        correction consume the dense device matrices directly.  One D2H of the corrected
        matrix at the end.  The corrected X keeps the input's float dtype (the
        reference's in-place ``Z_corr -= ...`` on the float32 matrix)."""
        from .models.harmony import moe_correct_expression
        from .ops import sparse as sops
        from .utils.anndata_lite import _take

        n = A.shape[0]
        cols = np.flatnonzero(hv)
        nh = int(cols.size)
        cmap = np.full(A.shape[1], -1, np.int32)
        cmap[cols] = np.arange(nh, dtype=np.int32)
        rs = target_sum / _nonzero(sops.row_sums(A))
        f64 = ad.X.dtype == np.float64
        # host dtypes: normalize_total -> float32 unless float64; scale of integer -> float64
        norm_dt = torch.float64 if f64 else torch.float32
        raw_dt = torch.float64 if (f64 or np.issubdtype(ad.X.dtype, np.integer)) else torch.float32

        def scaled(row_scale, out_dtype):
            # stdscale_quantile_celing of the (normalised) HVG subset, densified
            xf = dict(row_scale=row_scale, col_map=cmap,
                      round_mid=row_scale is not None and out_dtype == torch.float32)
            _, var = sops.mean_var(A, ddof=1, n_out=nh, **xf)
            std = torch.sqrt(var)
            std[std == 0] = 1.0
            mv = float("inf") if max_scaled_thresh is None else float(max_scaled_thresh)
            if quantile_thresh is not None:
                vals = sops.transform(A, col_div=std, max_value=mv, out_dtype=out_dtype, **xf)
                thr = sops.quantile_with_zeros(vals, n * nh, quantile_thresh)
                del vals
                if out_dtype == torch.float32:
                    thr = float(np.float32(thr))
                mv = min(mv, thr)
            return sops.densify(A, n_out=nh, col_div=std, max_value=mv, out_dtype=out_dtype, **xf)

        anorm = scaled(rs, norm_dt)
        if makeplots:
            make_count_hist(AnnData(X=anorm[:1000].cpu().numpy()), num_cells=1000)
        X_pca = pp.pca_tensor(anorm, 50, zero_center=True)[0]
        if normalize_librarysize:
            src = anorm
        else:
            del anorm
            src = scaled(None, raw_dt)
        res = run_harmony(X_pca, ad.obs, harmony_vars, max_iter_harmony=max_iter_harmony,
                          theta=theta, device=src.device, init_backend="device")
        self.harmony_info_ = {"iterations": len(res.kmeans_rounds),
                              "kmeans_rounds": [int(r) + 1 for r in res.kmeans_rounds],
                              "max_iter_harmony": int(max_iter_harmony)}
        Xc = moe_correct_expression(src, res._R_t, res._Phi_moe_t, res._lamb_t, K=res.K,
                                    levels=res._lv)
        del src
        Xc.clamp_(min=0)
        out = AnnData(X=to_host(Xc), obs=ad.obs, var=ad.var.iloc[cols],
                      obsm=dict(ad.obsm),
                      varm={k: (v[cols] if not isinstance(v, pd.DataFrame) else v.iloc[cols])
                            for k, v in ad.varm.items()},
                      layers={k: _take(v, slice(None), cols) for k, v in ad.layers.items()},
                      uns=dict(ad.uns))
        out.obsm["X_pca"] = X_pca
        out.obsm["X_pca_harmony"] = res.Z_corr.T
        return out

    def harmony_correct_X(self, X, obs, pca, harmony_vars, theta=1, max_iter_harmony=20,
                          device=None, init_backend=None):
        """Harmony on the PCs, then the MOE ridge correction applied to the expression
        matrix itself, clamped at 0 (preprocess.py:342-388).  Returns (X_corr, X_pca_harmony)."""
        dev = torch.device(device) if device is not None else _default_device()
        if init_backend is None:   # harmonypy's sklearn KMeans init on CPU; k-means on the GPU
            init_backend = "device" if dev.type == "cuda" else "sklearn"
        res = run_harmony(pca, obs, harmony_vars, max_iter_harmony=max_iter_harmony, theta=theta,
                          device=dev, init_backend=init_backend)
        self.harmony_info_ = {"iterations": len(res.kmeans_rounds),
                              "kmeans_rounds": [int(r) + 1 for r in res.kmeans_rounds],
                              "max_iter_harmony": int(max_iter_harmony)}
        X_pca_harmony = res.Z_corr.T
        _, X_corr, _, _ = moe_correct_ridge(np.asarray(X).T, None, None, res.R, None, res.K, None,
                                            res.Phi_moe, res.lamb, device=dev)
        X_corr = np.array(X_corr.T)
        X_corr[X_corr < 0] = 0
        return X_corr, X_pca_harmony

    def select_features_MI(self, _adata, cluster, max_scaled_thresh=None, quantile_thresh=.9999,
                           n_top_features=70, makeplots=True):
        """Mutual-information feature ranking against cluster labels (preprocess.py:391-439)."""
        from sklearn.feature_selection import mutual_info_classif

        ad = pp.normalize_total(to_lite(_adata))
        ad = stdscale_quantile_celing(ad, max_value=max_scaled_thresh,
                                      quantile_thresh=quantile_thresh)
        Xd = ad.X.toarray() if sp.issparse(ad.X) else ad.X
        res = mutual_info_classif(Xd, cluster, discrete_features="auto", n_neighbors=3, copy=True,
                                  random_state=self.random_seed)
        res = pd.Series(res, index=ad.var.index).sort_values(ascending=False)
        resdf = pd.DataFrame([res.values, np.arange(res.shape[0])], columns=res.index,
                             index=["MI", "MI_Rank"]).T
        resdf["MI_diff"] = resdf["MI"].diff()
        if makeplots:
            from .utils.plotting import _plt

            plt = _plt()
            fig, ax = plt.subplots(1, 1, figsize=(10, 3), dpi=100)
            ax.scatter(resdf["MI_Rank"], resdf["MI"])
            ax.set_ylabel("MI", fontsize=11)
            ax.set_xlabel("MI Rank", fontsize=11)
            ylim = ax.get_ylim()
            ax.vlines(x=n_top_features, ymin=ylim[0], ymax=ylim[1], linestyle="--", color="k")
            ax.set_ylim(ylim)
        for v in resdf.columns:
            ad.var[v] = resdf[v].reindex(ad.var.index).values
        ad.var["highly_variable"] = ad.var["MI_Rank"] < n_top_features
        return ad


def _nonzero(t: torch.Tensor) -> torch.Tensor:
    """normalize_total's guard: zero-count cells are divided by 1 (stay zero)."""
    return t + (t == 0)


def _device_counts(ad, dev):
    """The counts of ``ad`` as a device CSR when the device pipeline applies (GPU and a
    sparse matrix), else None."""
    if dev.type != "cuda" or not sp.issparse(ad.X):
        return None
    from .ops import sparse as sops

    return sops.DeviceCSR.from_scipy(ad.X, device=dev)


def _is_anndata(o) -> bool:
    return hasattr(o, "X") and hasattr(o, "obs") and hasattr(o, "var")

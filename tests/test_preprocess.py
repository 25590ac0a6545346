"""Preprocess / Harmony / h5ad / scanpy-equivalent helpers (C30-C38).

harmonypy and scanpy are not installed in this environment, so Harmony is checked on its
defining properties (objective decreases, batch structure is removed from the corrected
PCs, deterministic for a seed) -- parity with harmonypy itself is unpinned.
"""
import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sp
import torch

from cnmf_torch_amd import Preprocess
from cnmf_torch_amd.models import pp
from cnmf_torch_amd.models.harmony import moe_correct_ridge, run_harmony
from cnmf_torch_amd.utils.anndata_lite import AnnData
from cnmf_torch_amd.utils.h5ad import read_h5ad, write_h5ad
from cnmf_torch_amd.utils.synthetic import simulate_counts


def _batched_pcs(n=600, d=10, n_batch=3, seed=0):
    rs = np.random.default_rng(seed)
    n_types = 3
    types = rs.integers(0, n_types, n)
    batch = rs.integers(0, n_batch, n)
    centers = rs.normal(size=(n_types, d)) * 3
    shifts = rs.normal(size=(n_batch, d)) * 2
    Z = centers[types] + shifts[batch] + 0.3 * rs.normal(size=(n, d))
    meta = pd.DataFrame({"batch": pd.Categorical([f"b{b}" for b in batch]),
                         "type": types})
    return Z, meta, types, batch


def _batch_separation(Z, batch):
    """Between-batch centroid spread relative to the total spread."""
    mu = Z.mean(0)
    cb = np.stack([Z[batch == b].mean(0) for b in np.unique(batch)])
    return float(np.linalg.norm(cb - mu, axis=1).mean() / np.linalg.norm(Z - mu, axis=1).mean())


def test_harmony_removes_batch_effect_and_is_deterministic():
    Z, meta, types, batch = _batched_pcs()
    res = run_harmony(Z, meta, "batch", max_iter_harmony=10, random_state=0)
    Zc = res.Z_corr.T
    assert Zc.shape == Z.shape
    assert _batch_separation(Zc, batch) < 0.7 * _batch_separation(Z, batch)
    # cell types stay separated
    assert _batch_separation(Zc, types) > 0.5 * _batch_separation(Z, types)
    obj = res.objective_harmony
    assert obj[-1] <= obj[0]
    assert res.R.shape == (res.K, Z.shape[0])
    np.testing.assert_allclose(res.R.sum(0), 1.0, rtol=1e-10)
    res2 = run_harmony(Z, meta, "batch", max_iter_harmony=10, random_state=0)
    np.testing.assert_allclose(res2.Z_corr, res.Z_corr, rtol=1e-10, atol=1e-12)  # threaded BLAS


def test_harmony_two_covariates():
    Z, meta, types, batch = _batched_pcs(n=450, n_batch=2, seed=3)
    meta["donor"] = pd.Categorical(np.random.default_rng(1).integers(0, 3, len(meta)).astype(str))
    res = run_harmony(Z, meta, ["batch", "donor"], max_iter_harmony=5, random_state=1)
    assert res.Phi.shape[0] == 2 + 3
    assert np.isfinite(res.Z_corr).all()


def test_moe_correct_ridge_matches_sequential_formula():
    """Batched ridge correction == the reference's per-cluster loop (preprocess.py:9-18)."""
    rs = np.random.default_rng(0)
    F, N, K, B = 7, 80, 4, 2
    Z = rs.random((F, N))
    R = rs.random((K, N))
    R /= R.sum(0)
    b = rs.integers(0, B, N)
    Phi = np.zeros((B, N))
    Phi[b, np.arange(N)] = 1
    Phi_moe = np.vstack([np.ones((1, N)), Phi])
    lamb = np.diag([0.0, 1.0, 1.0])
    Zc = Z.copy()
    for i in range(K):
        Phi_Rk = Phi_moe * R[i]
        x = Phi_Rk @ Phi_moe.T + lamb
        W = np.linalg.inv(x) @ Phi_Rk @ Z.T
        W[0, :] = 0
        Zc -= W.T @ Phi_Rk
    Zcos = Zc / np.linalg.norm(Zc, ord=2, axis=0)
    got_cos, got_corr, W_last, Phi_Rk_last = moe_correct_ridge(Z, None, None, R, None, K, None,
                                                                Phi_moe, lamb)
    np.testing.assert_allclose(got_corr, Zc, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(got_cos, Zcos, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(W_last, W, rtol=1e-10, atol=1e-12)


def test_h5ad_roundtrip(tmp_path):
    rs = np.random.default_rng(0)
    X = sp.random(40, 25, density=0.3, format="csr", random_state=1, dtype=np.float32)
    obs = pd.DataFrame({"batch": pd.Categorical(rs.choice(["a", "b"], 40)),
                        "n": rs.integers(0, 9, 40), "ok": rs.random(40) > 0.5,
                        "score": rs.random(40)}, index=[f"c{i}" for i in range(40)])
    var = pd.DataFrame({"gene_ids": [f"ENSG{i}" for i in range(25)],
                        "highly_variable": rs.random(25) > 0.5},
                       index=[f"g{i}" for i in range(25)])
    ad = AnnData(X=X, obs=obs, var=var)
    ad.obsm["X_pca"] = rs.random((40, 3))
    fn = str(tmp_path / "t.h5ad")
    write_h5ad(fn, ad)
    back = read_h5ad(fn)
    assert sp.issparse(back.X)
    np.testing.assert_array_equal(back.X.toarray(), X.toarray())
    pd.testing.assert_index_equal(back.obs.index, obs.index)
    assert list(back.obs["batch"].astype(str)) == list(obs["batch"].astype(str))
    np.testing.assert_array_equal(back.obs["ok"].values.astype(bool), obs["ok"].values)
    np.testing.assert_allclose(back.obs["score"].values, obs["score"].values)
    np.testing.assert_array_equal(back.var["highly_variable"].values.astype(bool),
                                  var["highly_variable"].values)
    np.testing.assert_allclose(back.obsm["X_pca"], ad.obsm["X_pca"])
    dense = AnnData(X=X.toarray().astype(np.float64), obs=obs, var=var)
    write_h5ad(fn, dense)
    np.testing.assert_array_equal(read_h5ad(fn).X, dense.X)


def test_pp_scale_and_normalize_semantics():
    rs = np.random.default_rng(0)
    X = rs.poisson(2.0, (50, 8)).astype(np.float64)
    X[:, 3] = 5.0                                   # zero-variance gene stays unscaled
    ad = AnnData(X=X.copy())
    pp.scale(ad, zero_center=False)
    sd = X.std(axis=0, ddof=1)
    exp = X.copy()
    exp[:, sd > 0] /= sd[sd > 0]
    np.testing.assert_allclose(ad.X, exp)
    ad2 = pp.normalize_total(AnnData(X=X.copy()), target_sum=1e4, copy=True)
    np.testing.assert_allclose(ad2.X.sum(1), 1e4)
    Xs = sp.csr_matrix(X)
    ad3 = AnnData(X=Xs.copy())
    pp.scale(ad3, zero_center=False)
    np.testing.assert_allclose(ad3.X.toarray(), exp)


def test_preprocess_for_cnmf_with_and_without_harmony(tmp_path):
    Xc, cells, genes = simulate_counts(300, 120, 3, seed=2, sparse=True)
    rs = np.random.default_rng(0)
    obs = pd.DataFrame({"batch": pd.Categorical(rs.choice(["x", "y"], 300))}, index=cells)
    ad = AnnData(X=sp.csr_matrix(Xc), obs=obs, var=pd.DataFrame(index=genes))
    p = Preprocess(random_seed=0)
    filt = p.filter_adata(ad, min_cells_per_gene=3, min_counts_per_cell=10, makeplots=False)
    assert filt.shape[0] <= 300 and filt.shape[1] <= 120
    out, tp10k, hvgs = p.preprocess_for_cnmf(filt, n_top_rna_genes=40, makeplots=False,
                                             save_output_base=str(tmp_path / "pp"))
    assert len(hvgs) == 40 and out.shape[1] == 40
    np.testing.assert_allclose(np.asarray(tp10k.X.sum(1)).ravel(), 1e4, rtol=1e-6)
    assert (tmp_path / "pp.Corrected.HVG.Varnorm.h5ad").exists()
    out_h, _, _ = p.preprocess_for_cnmf(filt, harmony_vars="batch", n_top_rna_genes=40,
                                        makeplots=False, max_iter_harmony=3, device="cpu")
    Xh = out_h.X.toarray() if sp.issparse(out_h.X) else out_h.X
    assert Xh.shape == (filt.shape[0], 40) and (Xh >= 0).all()
    assert "X_pca_harmony" in out_h.obsm


def test_select_features_mi():
    Xc, cells, genes = simulate_counts(200, 60, 3, seed=5, sparse=False)
    labels = np.random.default_rng(0).integers(0, 3, 200)
    ad = AnnData(X=Xc.astype(np.float64), var=pd.DataFrame(index=genes),
                 obs=pd.DataFrame(index=cells))
    out = Preprocess(random_seed=0).select_features_MI(ad, labels, n_top_features=10,
                                                       makeplots=False)
    assert out.var["highly_variable"].sum() == 10
    assert {"MI", "MI_Rank", "MI_diff"} <= set(out.var.columns)


def test_pca_matches_sklearn():
    from sklearn.decomposition import PCA

    rs = np.random.default_rng(0)
    X = rs.normal(size=(300, 40)) @ rs.normal(size=(40, 40)) + rs.normal(size=40)
    ad = pp.pca(AnnData(X=X.copy()), n_comps=10)
    ref = PCA(n_components=10, svd_solver="full").fit(X)
    Z = ref.transform(X)
    got = ad.obsm["X_pca"]
    # same subspace and scores up to per-component sign
    for j in range(10):
        s = np.sign(np.dot(got[:, j], Z[:, j]))
        np.testing.assert_allclose(got[:, j] * s, Z[:, j], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(ad.uns["pca"]["variance"], ref.explained_variance_, rtol=1e-8)


def test_quantile_ceiling_sparse_matches_dense():
    from cnmf_torch_amd.preprocess import stdscale_quantile_celing

    rs = np.random.default_rng(2)
    X = rs.poisson(0.4, (400, 60)).astype(np.float64)
    for q in (0.9, 0.999, 0.5):
        a = stdscale_quantile_celing(AnnData(X=sp.csr_matrix(X)), quantile_thresh=q)
        b = stdscale_quantile_celing(AnnData(X=X.copy()), quantile_thresh=q)
        np.testing.assert_allclose(a.X.toarray(), b.X, rtol=1e-12, atol=1e-12)


def test_moe_correct_expression_matches_ridge():
    """Device-resident (cells x features) MOE correction == preprocess.py:9-18 formula."""
    from cnmf_torch_amd.models.harmony import moe_correct_expression

    rs = np.random.default_rng(1)
    F, N, K, B = 6, 90, 3, 3
    X = rs.random((N, F))
    R = rs.random((K, N))
    R /= R.sum(0)
    b = rs.integers(0, B, N)
    Phi = np.zeros((B, N))
    Phi[b, np.arange(N)] = 1
    Phi_moe = np.vstack([np.ones((1, N)), Phi])
    lamb = np.diag([0.0] + [1.0] * B)
    _, Zc, _, _ = moe_correct_ridge(X.T, None, None, R, None, K, None, Phi_moe, lamb)
    got = moe_correct_expression(torch.from_numpy(X), R, Phi_moe, lamb, K=K, chunk=32)
    np.testing.assert_allclose(got.numpy(), Zc.T, rtol=1e-10, atol=1e-12)
    got32 = moe_correct_expression(torch.from_numpy(X.astype(np.float32)), R, Phi_moe, lamb)
    assert got32.dtype == torch.float32


@pytest.mark.gpu
def test_device_harmony_pipeline_matches_host():
    """normalize_batchcorrect(harmony) with the counts resident on the GPU (fused CSR
    kernels) selects the same HVGs and produces the same PCs as the host pipeline."""
    Xc, cells, genes = simulate_counts(3000, 400, 4, seed=3, sparse=True)
    rs = np.random.default_rng(0)
    obs = pd.DataFrame({"batch": pd.Categorical(rs.choice(["x", "y", "z"], 3000))}, index=cells)
    ad = AnnData(X=sp.csr_matrix(Xc, dtype=np.float32), obs=obs, var=pd.DataFrame(index=genes))
    p = Preprocess(random_seed=0)
    d_out, d_hv = p.normalize_batchcorrect(ad.copy(), harmony_vars=["batch"], n_top_genes=100,
                                           makeplots=False, max_iter_harmony=3, device="cuda")
    h_out, h_hv = p.normalize_batchcorrect(ad.copy(), harmony_vars=["batch"], n_top_genes=100,
                                           makeplots=False, max_iter_harmony=3, device="cpu")
    assert d_hv == h_hv
    np.testing.assert_allclose(d_out.obsm["X_pca"], h_out.obsm["X_pca"], rtol=1e-4, atol=1e-4)
    assert d_out.X.shape == (3000, 100) and d_out.X.dtype == np.float32
    assert (d_out.X >= 0).all() and np.isfinite(d_out.X).all()
    # TP10K from the device matches the host normalisation (to one float32 ulp: the
    # device sums a cell's counts in float64, scipy in float32)
    _, tp_d, _ = p.preprocess_for_cnmf(ad.copy(), harmony_vars=["batch"], n_top_rna_genes=100,
                                       makeplots=False, max_iter_harmony=2, device="cuda")
    tp_h = pp.normalize_total(ad.copy(), target_sum=1e4, copy=True)
    np.testing.assert_allclose(tp_d.X.toarray(), tp_h.X.toarray(), rtol=2.5e-7, atol=0)

"""Device CSR preprocessing ops (ops/sparse.py, csrc/kernels/sparse.hip).

CPU: the torch paths against numpy / scipy / sklearn semantics (the host pipeline of
models/pp.py).  GPU: the HIP kernels against those torch paths -- bitwise where the
operation order is the same, to float64 rounding for the reductions.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from cnmf_torch_amd.ops import sparse as sops


def _counts(n=300, m=70, density=0.2, seed=0, dtype=np.float32):
    rs = np.random.default_rng(seed)
    X = sp.random(n, m, density=density, format="csr", random_state=rs,
                  data_rvs=lambda k: rs.integers(1, 30, k)).astype(dtype)
    X[5] = 0            # an empty row
    X = X.tocsr()
    X.eliminate_zeros()
    X[:, 3] = 0         # an empty column
    X = X.tocsr()
    X.eliminate_zeros()
    return X


def _dev():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def test_row_sums_and_mean_var_match_sklearn():
    from sklearn.utils.sparsefuncs import mean_variance_axis

    X = _counts()
    A = sops.DeviceCSR.from_scipy(X)
    np.testing.assert_allclose(sops.row_sums(A).numpy(), np.asarray(X.sum(1)).ravel())
    mean, var = sops.mean_var(A)
    m_ref, v_ref = mean_variance_axis(X.astype(np.float64), axis=0)
    np.testing.assert_allclose(mean.numpy(), m_ref, rtol=1e-13)
    np.testing.assert_allclose(var.numpy(), v_ref, rtol=1e-12, atol=1e-14)
    _, var1 = sops.mean_var(A, ddof=1)
    np.testing.assert_allclose(var1.numpy(), v_ref * X.shape[0] / (X.shape[0] - 1), rtol=1e-12)


def test_transform_matches_host_pipeline():
    """normalize_total -> column subset -> scale(zero_center=False, max_value) in one pass
    equals the host CSR pipeline (same sparsity, values to one float32 ulp: the gene std
    comes from a different float64 summation order than sklearn's)."""
    from cnmf_torch_amd.models import pp
    from cnmf_torch_amd.utils.anndata_lite import AnnData

    X = _counts()
    ad = AnnData(X=X.copy())
    norm = pp.normalize_total(ad, target_sum=1e4, copy=True)
    keep = np.zeros(X.shape[1], bool)
    keep[::3] = True
    sub = norm[:, keep]
    host = pp.scale(sub, zero_center=False, max_value=4.0).X.tocsr()

    A = sops.DeviceCSR.from_scipy(X)
    rsum = sops.row_sums(A)
    rs = 1e4 / (rsum + (rsum == 0))
    cmap = np.full(X.shape[1], -1, np.int32)
    cmap[keep] = np.arange(keep.sum())
    _, var = sops.mean_var(A, ddof=1, row_scale=rs, col_map=cmap, n_out=int(keep.sum()),
                           round_mid=True)
    std = torch.sqrt(var)
    std[std == 0] = 1.0
    vals = sops.transform(A, row_scale=rs, col_map=cmap, col_div=std, max_value=4.0,
                          round_mid=True)
    got = vals[vals >= 0].numpy()
    np.testing.assert_allclose(got, host.data, rtol=3e-7, atol=0)
    D = sops.densify(A, n_out=int(keep.sum()), row_scale=rs, col_map=cmap, col_div=std,
                     max_value=4.0, round_mid=True)
    np.testing.assert_allclose(D.numpy(), host.toarray(), rtol=3e-7, atol=0)


def test_quantile_with_zeros_matches_numpy():
    rs = np.random.default_rng(3)
    vals = rs.random(1000).astype(np.float32) * 10
    vals[::7] = -1.0                       # dropped entries
    n_total = 5000
    stored = vals[vals >= 0]
    full = np.concatenate([np.zeros(n_total - stored.size, np.float32), stored])
    for q in (0.5, 0.9, 0.9999, 0.0, 1.0):
        got = sops.quantile_with_zeros(torch.from_numpy(vals), n_total, q)
        assert got == pytest.approx(float(np.quantile(full, q)), rel=1e-6, abs=1e-7)


def test_col_stats_clip_matches_numpy():
    X = _counts(seed=2)
    clip = np.linspace(1, 20, X.shape[1])
    A = sops.DeviceCSR.from_scipy(X)
    s, q, k = sops.col_stats(A, clip=clip)
    Xc = X.astype(np.float64).copy()
    Xc.data = np.minimum(Xc.data, clip[Xc.indices])
    np.testing.assert_allclose(s.numpy(), np.asarray(Xc.sum(0)).ravel(), rtol=1e-13)
    np.testing.assert_allclose(q.numpy(), np.asarray(Xc.multiply(Xc).sum(0)).ravel(), rtol=1e-13)
    np.testing.assert_array_equal(k.numpy(), np.diff(X.tocsc().indptr))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("m", [70, 4000])
def test_sparse_kernels_match_torch(dtype, m):
    X = _counts(n=2500, m=m, density=0.05 if m > 1000 else 0.2, seed=m, dtype=dtype)
    Ac = sops.DeviceCSR.from_scipy(X)
    Ag = sops.DeviceCSR.from_scipy(X, device="cuda")
    torch.testing.assert_close(sops.row_sums(Ag).cpu(), sops.row_sums(Ac), rtol=1e-13, atol=0)
    rs = np.random.default_rng(0).random(X.shape[0]) + 0.5
    cmap = np.where(np.arange(m) % 4 == 1, -1, 0).astype(np.int32)
    cmap[cmap == 0] = np.arange((cmap == 0).sum())
    nout = int((cmap >= 0).sum())
    div = np.random.default_rng(1).random(nout) + 0.5
    clip = np.random.default_rng(2).random(nout) * 30
    xf = dict(row_scale=rs, col_map=cmap, n_out=nout, col_div=div, clip=clip, max_value=25.0,
              round_mid=True)
    for a, b in zip(sops.col_stats(Ag, **xf), sops.col_stats(Ac, **xf)):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-12, atol=1e-12)
    mg, vg = sops.mean_var(Ag, ddof=1, **xf)
    mc, vc = sops.mean_var(Ac, ddof=1, **xf)
    torch.testing.assert_close(mg.cpu(), mc, rtol=1e-12, atol=1e-14)
    torch.testing.assert_close(vg.cpu(), vc, rtol=1e-10, atol=1e-13)
    # determinism
    assert torch.equal(sops.col_stats(Ag, **xf)[1], sops.col_stats(Ag, **xf)[1])
    xf.pop("n_out")
    for od in (torch.float32, torch.float64):
        assert torch.equal(sops.transform(Ag, out_dtype=od, **xf).cpu(),
                           sops.transform(Ac, out_dtype=od, **xf))
        assert torch.equal(sops.densify(Ag, n_out=nout, out_dtype=od, **xf).cpu(),
                           sops.densify(Ac, n_out=nout, out_dtype=od, **xf))
    vals = sops.transform(Ag, **xf)
    n_total = X.shape[0] * nout
    for q in (0.5, 0.99, 0.9999):
        assert sops.quantile_with_zeros(vals, n_total, q) == \
            sops.quantile_with_zeros(vals.cpu(), n_total, q)


def test_spmm_tspmm_views_match_dense():
    """CSR products through a lazy scaled-subset view == dense numpy on the same matrix."""
    X = _counts(n=400, m=90, seed=4)
    A = sops.DeviceCSR.from_scipy(X)
    hv = np.array([5, 1, 40, 7, 88, 60])                 # unsorted subset, like an HVG list
    cmap = np.full(X.shape[1], -1, np.int32)
    cmap[hv] = np.arange(hv.size)
    std = np.random.default_rng(0).random(hv.size) + 0.5
    V = A.view(col_map=cmap, col_div=std, n_out=hv.size)
    assert V.shape == (400, hv.size)
    D = (X[:, hv].toarray().astype(np.float64) / std).astype(np.float32)
    np.testing.assert_array_equal(sops.densify(V).numpy(), D)
    B = np.random.default_rng(1).random((hv.size, 7)).astype(np.float32)
    np.testing.assert_allclose(sops.spmm(V, torch.from_numpy(B)).numpy(), D @ B, rtol=1e-5)
    U = np.random.default_rng(2).random((400, 7))
    np.testing.assert_allclose(sops.tspmm(V, torch.from_numpy(U)).numpy(),
                               D.astype(np.float64).T @ U, rtol=1e-6)
    np.testing.assert_allclose(sops.tspmm(A, torch.from_numpy(U)).numpy(),
                               X.toarray().astype(np.float64).T @ U, rtol=1e-12)


def test_refit_and_ols_accept_device_csr():
    from cnmf_torch_amd.models.ols import efficient_ols_all_cols
    from cnmf_torch_amd.models.refit import fit_H_online, fit_spectra_online

    X = _counts(n=500, m=60, seed=6)
    A = sops.DeviceCSR.from_scipy(X)
    W = np.random.default_rng(0).random((4, 60))
    h1 = fit_H_online(X, W, chunk_size=128, random_state=3)
    h2 = fit_H_online(A, W, chunk_size=128, random_state=3)
    np.testing.assert_allclose(h2, h1, rtol=1e-4, atol=1e-6)
    U = np.random.default_rng(1).random((500, 4))
    s1 = fit_spectra_online(X, U, chunk_size=32, random_state=3)
    s2 = fit_spectra_online(A, U, chunk_size=32, random_state=3)
    np.testing.assert_allclose(s2, s1, rtol=1e-4, atol=1e-6)
    b1 = efficient_ols_all_cols(U, X, normalize_y=True)
    b2 = efficient_ols_all_cols(U, A, normalize_y=True)
    # StandardScaler keeps float32 input in float32 for the z-score statistics; the CSR
    # path accumulates them in float64
    np.testing.assert_allclose(b2, b1, rtol=1e-5, atol=1e-9)
    b3 = efficient_ols_all_cols(U, X.astype(np.float64), normalize_y=True)
    np.testing.assert_allclose(b2, b3, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [3, 10, 40])
def test_spmm_tspmm_kernels_match_torch(K):
    X = _counts(n=3000, m=2500, density=0.03, seed=K)
    Ac = sops.DeviceCSR.from_scipy(X)
    Ag = sops.DeviceCSR.from_scipy(X, device="cuda")
    cmap = np.where(np.arange(2500) % 3 == 0, -1, 0).astype(np.int32)
    cmap[cmap == 0] = np.random.default_rng(K).permutation(int((cmap == 0).sum()))
    nout = int((cmap >= 0).sum())
    std = np.random.default_rng(0).random(nout) + 0.5
    xf = dict(col_map=cmap, col_div=std, n_out=nout)
    Vc, Vg = Ac.view(**xf), Ag.view(**xf)
    B = torch.rand((nout, K))
    torch.testing.assert_close(sops.spmm(Vg, B.cuda()).cpu(), sops.spmm(Vc, B), rtol=1e-5,
                               atol=1e-5)
    U = torch.rand((3000, K), dtype=torch.float64)
    got = sops.tspmm(Vg, U.cuda())
    torch.testing.assert_close(got.cpu(), sops.tspmm(Vc, U), rtol=1e-12, atol=1e-12)
    assert torch.equal(got, sops.tspmm(Vg, U.cuda()))          # deterministic
    torch.testing.assert_close(sops.tspmm(Ag, U.float().cuda()).cpu(),
                               sops.tspmm(Ac, U.float()), rtol=1e-12, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse_tpm", [True, False])
def test_norm_counts_dense_device_matches_host(sparse_tpm, tmp_path, monkeypatch):
    """get_norm_counts on a dense count matrix: GPU gather+scale == host numpy path."""
    import pandas as pd

    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.utils.anndata_lite import AnnData

    rs = np.random.default_rng(0)
    X = rs.poisson(2.0, (800, 120)).astype(np.float32)
    X[:, 7] = 3.0                                   # constant gene
    counts = AnnData(X=X, obs=pd.DataFrame(index=[f"c{i}" for i in range(800)]),
                     var=pd.DataFrame(index=[f"g{j}" for j in range(120)]))
    tpm = AnnData(X=sp.csr_matrix(X) if sparse_tpm else X.copy(), obs=counts.obs, var=counts.var)
    genes = [f"g{j}" for j in (5, 7, 90, 3, 44)]
    obj = cNMF(output_dir=str(tmp_path), name="nc")
    got = obj.get_norm_counts(counts, tpm, high_variance_genes_filter=genes)
    monkeypatch.setenv("CNMF_DEVICE", "cpu")
    ref = obj.get_norm_counts(counts, tpm, high_variance_genes_filter=genes)
    assert list(got.var.index) == genes
    np.testing.assert_allclose(got.X, ref.X, rtol=1e-12, atol=0, equal_nan=True)


def test_gemm_plan_fills_whole_waves_for_mid_size_batches():
    """ops.gemm_plan: K x replicates in (1024, 4096] takes 128 x 256 tiles with the k split
    that best fills whole waves of CUs (profiles/r4q_gemm_plan_sweep.json.log); the K = 10
    and K = 50 shapes keep the measured plans of earlier rounds."""
    from cnmf_torch_amd import ops

    assert ops.gemm_plan(1000, 5000, 2048, 1) == (4, 1)      # K=10 numerator
    assert ops.gemm_plan(1000, 2000, 5056, 1) == (1, 4)      # K=10 statistics
    assert ops.gemm_plan(2000, 5000, 2048, 1) == (1, 2)      # K=20 numerator: 320 tiles
    assert ops.gemm_plan(2000, 2000, 5056, 1) == (1, 2)      # K=20 statistics
    assert ops.gemm_plan(3000, 5000, 2048, 1) == (1, 1)      # K=30 numerator
    assert ops.gemm_plan(5000, 5000, 2048, 1) == (1, 1)      # K=50: the older rule


@pytest.mark.gpu
def test_from_scipy_canonical_check_on_device():
    """An unchecked CSR is checked for sorted, distinct columns (scipy's check, on a
    worker thread while the arrays upload); one that is not canonical is summed on the
    host like scipy's own path -- the device result is canonical either way."""
    m = sp.random(300, 120, density=0.1, format="csr", random_state=1, dtype=np.float32)
    for case in ("sorted", "reversed", "duplicate"):
        ind = m.indices.copy()
        data = m.data.copy()
        if case == "reversed":
            for r in range(m.shape[0]):
                a, b = m.indptr[r], m.indptr[r + 1]
                ind[a:b] = ind[a:b][::-1].copy()
                data[a:b] = data[a:b][::-1].copy()
        elif case == "duplicate":
            r = int(np.flatnonzero(np.diff(m.indptr) >= 2)[0])
            ind[m.indptr[r] + 1] = ind[m.indptr[r]]
        x = sp.csr_matrix((data, ind, m.indptr.copy()), shape=m.shape)
        A = sops.DeviceCSR.from_scipy(x, device="cuda")
        assert sops._sorted_distinct(A)
        ref = x.copy()
        ref.sum_duplicates()
        np.testing.assert_array_equal(A.to_scipy().toarray(), ref.toarray())
        np.testing.assert_array_equal(A.indptr.cpu().numpy(), ref.indptr)

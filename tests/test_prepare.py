"""Port of the reference's prepare tests (tests/test_prepare.py:61-96) onto our engine:
3 formats x 3 dtypes x dense/sparse, plus the zero-HVG-cell guard."""
import os

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sp

from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
from cnmf_torch_amd.utils.anndata_lite import AnnData
from cnmf_torch_amd.utils.h5ad import read_h5ad

NUM_CELLS, NUM_GENES, SEED = 100, 500, 42


def _counts_file(tmp_path, fmt, dtype, zero_count=False):
    np.random.seed(SEED)
    data = np.random.binomial(n=100, p=0.01, size=(NUM_CELLS, NUM_GENES)).astype(dtype)
    if zero_count:
        data[0, :] = 0
    cells = [f"cell{i}" for i in range(NUM_CELLS)]
    genes = [f"gene{i}" for i in range(NUM_GENES)]
    if fmt == "txt":
        fn = tmp_path / f"counts_{dtype.__name__}.txt"
        pd.DataFrame(data, index=cells, columns=genes).to_csv(fn, sep="\t")
    elif fmt == "npz":
        fn = tmp_path / f"counts_{dtype.__name__}.npz"
        save_df_to_npz(pd.DataFrame(data, index=cells, columns=genes), str(fn))
    else:
        fn = tmp_path / f"counts_{dtype.__name__}.h5ad"
        AnnData(X=sp.csr_matrix(data)).write_h5ad(str(fn))
    return str(fn)


@pytest.mark.parametrize("fmt", ["txt", "npz", "h5ad"])
@pytest.mark.parametrize("dtype", [np.int64, np.float32, np.float64])
@pytest.mark.parametrize("densify", [True, False])
def test_prepare(tmp_path, fmt, dtype, densify):
    obj = cNMF(output_dir=str(tmp_path), name="test")
    obj.prepare(_counts_file(tmp_path, fmt, dtype), components=[5, 10], n_iter=10, densify=densify)
    for key in ("normalized_counts", "nmf_replicate_parameters", "nmf_run_parameters",
                "nmf_genes_list", "tpm", "tpm_stats"):
        assert os.path.exists(obj.paths[key]), key
    nc = read_h5ad(obj.paths["normalized_counts"])
    assert nc.shape[0] == NUM_CELLS and nc.X.dtype == np.float64
    ledger = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    assert list(ledger.columns) == ["n_components", "iter", "nmf_seed", "completed"]
    assert len(ledger) == 20


@pytest.mark.parametrize("fmt", ["txt", "npz", "h5ad"])
@pytest.mark.parametrize("densify", [True, False])
def test_prepare_raises_on_zero_count_cells(tmp_path, fmt, densify):
    obj = cNMF(output_dir=str(tmp_path), name="test")
    fn = _counts_file(tmp_path, fmt, np.int64, zero_count=True)
    with pytest.raises(Exception, match="Error: .* cells have zero counts of overdispersed genes.*"):
        obj.prepare(fn, components=[5, 10], n_iter=10, densify=densify)


def test_ledger_seeds_numpy_exact(tmp_path):
    """Seeds are numpy-legacy exact (seed 14, 45 runs)."""
    obj = cNMF(output_dir=str(tmp_path), name="t")
    rp, kw = obj.get_nmf_iter_params(ks=[5, 6, 7], n_iter=15, random_state_seed=14)
    assert rp["nmf_seed"].tolist()[:3] == [59886188, 1812018521, 1173234957]
    assert rp["n_components"].tolist() == [5] * 15 + [6] * 15 + [7] * 15
    assert kw["algo"] == "mu" and kw["mode"] == "online" and kw["tol"] == 1e-4
    for key in ("alpha_W", "alpha_H", "l1_ratio_H", "l1_ratio_W", "beta_loss", "online_chunk_max_iter",
                "online_chunk_size", "init", "n_jobs", "use_gpu"):
        assert key in kw


def test_norm_counts_semantics(tmp_path):
    """HVG subset of raw counts / ddof=1 std; TPM stats ddof=0 (cnmf.py:570-580, 670-681)."""
    fn = _counts_file(tmp_path, "npz", np.float64)
    obj = cNMF(output_dir=str(tmp_path), name="t")
    obj.prepare(fn, components=[5], n_iter=2, num_highvar_genes=50)
    raw = load_df_from_npz(fn)
    genes = open(obj.paths["nmf_genes_list"]).read().split("\n")
    assert len(genes) == 50
    nc = read_h5ad(obj.paths["normalized_counts"])
    X = nc.X.toarray()
    ref = raw[genes].values / raw[genes].values.std(axis=0, ddof=1)
    np.testing.assert_allclose(X, ref, rtol=1e-10)
    tpm = raw.values / raw.values.sum(axis=1, keepdims=True) * 1e6
    st = load_df_from_npz(obj.paths["tpm_stats"])
    np.testing.assert_allclose(st["__mean"].values, tpm.mean(axis=0), rtol=1e-5)
    np.testing.assert_allclose(st["__std"].values, tpm.std(axis=0, ddof=0), rtol=1e-4)


def test_sparse_mean_var_matches_sklearn_bitwise():
    """models.hvg.sparse_mean_var (no sklearn import on the prepare path) == the
    StandardScaler(with_mean=False) statistics cnmf.py:128-131 computes, bit for bit,
    for float32 / float64 / int64 CSR inputs, incl. a fully dense and an empty column."""
    import scipy.sparse as sp
    from sklearn.preprocessing import StandardScaler

    from cnmf_torch_amd.models.hvg import sparse_mean_var

    rng = np.random.default_rng(3)
    for dt in (np.float32, np.float64, np.int64):
        X = sp.random(2000, 300, density=0.1, random_state=2, format="lil")
        X[:, 7] = 3
        X[:, 11] = 0
        X = sp.csr_matrix(X)
        X.data = (rng.poisson(3, X.nnz) + 1) * (1.0 if dt == np.int64 else 1.37)
        X = X.astype(dt)
        m, v = sparse_mean_var(X)
        sc = StandardScaler(with_mean=False).fit(X)
        np.testing.assert_array_equal(m, sc.mean_)
        np.testing.assert_array_equal(v, sc.var_)

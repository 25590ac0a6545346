"""GPU pipeline pieces: the solver's early hand-over of retired replicates
(NMFBatchSolver.run(on_retire=...)) and the device-streamed norm counts of prepare."""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
from cnmf_torch_amd.utils.synthetic import simulate_counts

pytestmark = pytest.mark.gpu


def test_retired_replicates_handed_over_equal_final_spectra():
    """run(on_retire=cb): every replicate a host compaction retires is handed over once
    (pinned spectra + event) while the rest still solve, and those spectra equal the
    final result rows bit for bit."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 400, n_programs=6, seed=4)).cuda()
    got = {}

    def cb(idx, kpos, host, ev):
        ev.synchronize()
        off = np.concatenate([[0], np.cumsum(kpos)[:-1]])
        for i, o, k in zip(idx, off, kpos):
            assert int(i) not in got
            got[int(i)] = host[o:o + k].clone()

    kk = [4] * 30 + [6] * 30
    res = NMFBatchSolver(X, NMFOptions(n_components=4, online_chunk_size=1000)).run(
        list(range(50, 110)), ks=kk, on_retire=cb)
    assert len(got) > 10
    for i, w in got.items():
        assert torch.equal(w, res.spectra(i).cpu())


def test_streamed_norm_counts_equal_get_norm_counts(tmp_path):
    """prepare on the GPU with dense counts streams the float64 norm counts from the device
    into the h5ad (api._save_norm_counts_streamed): X, obs, var, obsm and uns equal the
    public get_norm_counts(...) AnnData, bit for bit; the genes list is written too."""
    from cnmf_torch_amd.utils.anndata_lite import AnnData
    from cnmf_torch_amd.utils.h5ad import read_h5ad, write_h5ad

    X, cells, genes = simulate_counts(2100, 400, 5, seed=9, sparse=False)
    ad = AnnData(X=X.astype(np.float32), obs=pd.DataFrame({"grp": ["a", "b", "c"] * 700},
                                                          index=cells),
                 var=pd.DataFrame(index=genes),
                 obsm={"X_pca": np.random.default_rng(0).random((2100, 7))},
                 uns={"note": "kept"})
    fn = str(tmp_path / "counts.h5ad")
    write_h5ad(fn, ad)
    obj = cNMF(output_dir=str(tmp_path), name="s")
    obj.prepare(fn, components=[5], n_iter=3, seed=1, num_highvar_genes=150)
    got = read_h5ad(obj.paths["normalized_counts"])
    with open(obj.paths["nmf_genes_list"]) as fh:
        hv = fh.read().split("\n")
    from cnmf_torch_amd.utils.io import read_any

    tpm = read_h5ad(obj.paths["tpm"])
    ref = obj.get_norm_counts(read_any(fn), tpm, high_variance_genes_filter=hv)
    np.testing.assert_array_equal(np.asarray(got.X), np.asarray(ref.X))
    assert got.X.dtype == np.float64
    assert list(got.var.index) == list(ref.var.index) == hv
    pd.testing.assert_frame_equal(got.obs, ref.obs, check_dtype=False, check_categorical=False)
    np.testing.assert_array_equal(got.obsm["X_pca"], ad.obsm["X_pca"])
    assert got.uns["note"] == "kept"


def test_k_selection_with_dense_device_counts_over_several_ks(tmp_path):
    """Dense normalised counts stay device-resident across the Ks of k_selection_plot:
    the cached ||X||^2 (api._XSQ) is looked up by tensor identity for the second K on
    (a WeakKeyDictionary compared tensor keys with Tensor.__eq__ and raised there)."""
    X, cells, genes = simulate_counts(1200, 400, 5, seed=8, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), fn)
    obj = cNMF(output_dir=str(tmp_path), name="dk")
    obj.prepare(fn, components=[4, 5, 6], n_iter=8, seed=3, num_highvar_genes=300,
                densify=True, use_gpu=True, batch_size=400)
    obj.factorize(worker_i=0, total_workers=1, verbose=False)
    obj.combine()
    obj.k_selection_plot(close_fig=True)
    stats = load_df_from_npz(obj.paths["k_selection_stats"])
    assert list(stats["k"]) == [4, 5, 6]
    assert np.all(np.isfinite(stats["prediction_error"].values))


def _pipeline(tmp, fn, name, densify):
    obj = cNMF(output_dir=str(tmp), name=name)
    obj.prepare(fn, components=[4, 5], n_iter=6, seed=3, num_highvar_genes=300,
                use_gpu=True, batch_size=400, densify=densify)
    obj.factorize(worker_i=0, total_workers=1, verbose=False)
    obj.combine()
    obj.k_selection_plot(close_fig=True)
    obj.consensus(5, density_threshold=2.0, show_clustering=False)
    return obj


@pytest.mark.parametrize("densify", [False, True])
def test_resident_norm_counts_mirror_equals_file_reads(tmp_path, monkeypatch, densify):
    """prepare's GPU path leaves a device mirror of the norm counts it wrote
    (utils.resident); factorize, k_selection_plot and consensus in the same process read
    it instead of the file.  Every artifact equals the file-reading run bit for bit, the
    mirror is what the stages used, and a rewritten file invalidates it."""
    from cnmf_torch_amd.utils import resident

    X, cells, genes = simulate_counts(1300, 450, 5, seed=12, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), fn)
    resident.forget()
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", "0")
    a = _pipeline(tmp_path, fn, "file", densify)
    assert resident.recall(a.paths["normalized_counts"], "X32") is None
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", str(1 << 30))
    b = _pipeline(tmp_path, fn, "mirror", densify)
    # (a sparse norm-counts file is mirrored for factorize only: consensus runs CSR kernels)
    tag = "X32" if densify else "X32_factorize"
    Xr = resident.recall(b.paths["normalized_counts"], tag)
    assert Xr is not None and Xr.is_cuda
    from cnmf_torch_amd.utils.h5ad import read_h5ad

    Xf = read_h5ad(b.paths["normalized_counts"]).X
    Xf = Xf.toarray() if hasattr(Xf, "toarray") else np.asarray(Xf)
    np.testing.assert_array_equal(Xr.cpu().numpy(), Xf.astype(np.float32))
    for key, args in (("iter_spectra", (5, 2)), ("merged_spectra", (4,)),
                      ("consensus_spectra", (5, "2_0")), ("consensus_usages", (5, "2_0")),
                      ("gene_spectra_score", (5, "2_0")), ("k_selection_stats", None)):
        fa = a.paths[key] % args if args else a.paths[key]
        fb = b.paths[key] % args if args else b.paths[key]
        da, db = load_df_from_npz(fa), load_df_from_npz(fb)
        np.testing.assert_array_equal(da.values, db.values)
    # rewriting the file drops the mirror
    os.utime(b.paths["normalized_counts"], ns=(1, 1))
    assert resident.recall(b.paths["normalized_counts"], tag) is None
    resident.forget()

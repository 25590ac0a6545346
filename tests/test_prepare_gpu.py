"""Per-gene statistics of the prepare stage on the GPU (the
reference's column statistics: cnmf.py:128-131, 570-580, 660-681).  The exact integer
moments of a host matrix are formed on the device block by block (models.hvg
_device_moment_digits, csrc/kernels/exact_moments.hip) and must be the host digits bit for
bit -- the property that keeps a sharded prepare identical to the single-process one."""
import numpy as np
import pytest
import scipy.sparse as sp

import dist_workers as W
from test_distributed import _spawn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sparse,dt", [(True, np.float32), (True, np.float64),
                                       (False, np.float32)])
def test_device_moment_digits_equal_host_digits(monkeypatch, sparse, dt):
    from cnmf_torch_amd.models import hvg

    rng = np.random.default_rng(5)
    n, g = 20000, 700
    X = rng.poisson(0.3, (n, g)).astype(dt) * rng.gamma(2.0, 3.0, (n, 1)).astype(dt)
    X[:, 5] = 0
    X[7, 9] = dt(1e-40)          # below the exact window (2^-126): counted, not summed
    M = sp.csr_matrix(X) if sparse else X
    host = hvg.exact_moment_digits(M)
    before = hvg.DEVICE_MOMENT_BLOCKS
    monkeypatch.setattr(hvg, "_device_moment_digits",
                        lambda X_, d_, block_bytes=1 << 20, f=hvg._device_moment_digits:
                        f(X_, d_, block_bytes=1 << 20))       # several row blocks
    dev = hvg.exact_moment_digits(M, device="cuda")
    assert hvg.DEVICE_MOMENT_BLOCKS - before > 3
    np.testing.assert_array_equal(host[0], dev[0])
    np.testing.assert_array_equal(host[1], dev[1])
    assert host[2] == dev[2] == 1
    mh = hvg.exact_mean_var(M, 1)
    assert mh is None          # a value outside the window: callers use floating point
    X[7, 9] = 0
    M = sp.csr_matrix(X) if sparse else X
    a, b = hvg.exact_mean_var(M, 1), hvg.exact_mean_var(M, 1, device="cuda")
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_sharded_prepare_statistics_on_the_gpu_match_single_process(tmp_path):
    """Two ranks on the box's GPU (gloo collectives): each rank's gene moments run in
    exact_moments.hip, and the artifacts equal the single-process prepare's bit for bit."""
    from cnmf_torch_amd import cNMF, load_df_from_npz
    from cnmf_torch_amd.utils.anndata_lite import AnnData
    from cnmf_torch_amd.utils.h5ad import read_h5ad, write_h5ad
    from cnmf_torch_amd.utils.synthetic import simulate_counts
    import pandas as pd

    Xc, cells, genes = simulate_counts(600, 300, 4, seed=21, sparse=True)
    fn = str(tmp_path / "counts.h5ad")
    write_h5ad(fn, AnnData(X=Xc, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
    kw = dict(components=[3, 4], n_iter=3, seed=7, num_highvar_genes=120)
    _spawn(W.prepare_worker, 2, str(tmp_path), "sh", fn, dict(kw), timeout=200)
    for r in range(2):
        assert int(np.load(tmp_path / f"devblocks{r}.npy")[0]) >= 2   # TPM + HVG counts
    ser = cNMF(output_dir=str(tmp_path), name="se")
    ser.prepare(fn, **kw)
    sh = cNMF(output_dir=str(tmp_path), name="sh")
    assert open(sh.paths["nmf_genes_list"]).read() == open(ser.paths["nmf_genes_list"]).read()
    np.testing.assert_array_equal(load_df_from_npz(sh.paths["tpm_stats"]).values,
                                  load_df_from_npz(ser.paths["tpm_stats"]).values)
    for key in ("normalized_counts", "tpm"):
        a, b = read_h5ad(sh.paths[key]), read_h5ad(ser.paths[key])
        xa = a.X.toarray() if hasattr(a.X, "toarray") else a.X
        xb = b.X.toarray() if hasattr(b.X, "toarray") else b.X
        np.testing.assert_array_equal(xa, xb)

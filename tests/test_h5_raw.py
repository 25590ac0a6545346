"""Raw parallel I/O of large contiguous h5ad matrices (csrc/h5ad/h5io.cpp raw_io): a
matrix written through the raw path reads back bit for bit through HDF5's own reader
and through the raw reader, row blocks land at their rows, sliced reads take the right
rows, and small / compressed / bool datasets keep the HDF5 path."""
import numpy as np
import pandas as pd

from cnmf_torch_amd.utils.anndata_lite import AnnData
from cnmf_torch_amd.utils.h5ad import (_lib, read_h5ad, read_X_row_segments, write_h5ad,
                                       write_h5ad_row_blocks)


def _ad(X):
    return AnnData(X=X, obs=pd.DataFrame(index=[f"c{i}" for i in range(X.shape[0])]),
                   var=pd.DataFrame(index=[f"g{i}" for i in range(X.shape[1])]))


def test_raw_write_read_roundtrip(tmp_path, monkeypatch):
    rng = np.random.default_rng(0)
    X = rng.random((9000, 1000))                 # 72 MB float64: the raw path
    p = str(tmp_path / "a.h5ad")
    write_h5ad(p, _ad(X))
    np.testing.assert_array_equal(read_h5ad(p).X, X)
    with _lib().File(p, "r") as f:               # rows through the raw reader
        np.testing.assert_array_equal(f.read("/X", 1234, 8800), X[1234:8800])
    # HDF5's own reader sees the same matrix (the raw bytes are the dataset's), and a
    # file HDF5 wrote itself reads back through the raw reader
    monkeypatch.setenv("CNMF_H5_RAW", "0")
    np.testing.assert_array_equal(read_h5ad(p).X, X)
    q = str(tmp_path / "h.h5ad")
    write_h5ad(q, _ad(X))
    monkeypatch.setenv("CNMF_H5_RAW", "1")
    np.testing.assert_array_equal(read_h5ad(q).X, X)
    segs = [(10, 4000), (5000, 8999)]
    np.testing.assert_array_equal(read_X_row_segments(p, segs),
                                  np.concatenate([X[10:4000], X[5000:8999]]))


def test_raw_row_blocks_and_small_arrays(tmp_path):
    rng = np.random.default_rng(1)
    X = rng.random((9000, 1000)).astype(np.float64)
    ad = _ad(X)

    def blocks():
        for a in range(0, X.shape[0], 4096):      # 32 MB blocks: below and above the cut
            yield None, X[a:a + 4096]

    p = str(tmp_path / "b.h5ad")
    write_h5ad_row_blocks(p, X.shape[0], ad.var, blocks(), sparse=False, dtype=np.float64,
                          obs=ad.obs)
    np.testing.assert_array_equal(read_h5ad(p).X, X)
    small = rng.random((50, 40)).astype(np.float32)
    q = str(tmp_path / "c.h5ad")
    write_h5ad(q, _ad(small), compression="gzip")
    np.testing.assert_array_equal(read_h5ad(q).X, small)

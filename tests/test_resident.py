"""utils.resident: device/host mirrors of files this process wrote are returned only
while the file is unchanged, and stay within the byte budget."""
import os

import numpy as np

from cnmf_torch_amd.utils import resident


def test_recall_only_while_file_unchanged(tmp_path, monkeypatch):
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", "1000000")
    resident.forget()
    p = tmp_path / "a.bin"
    p.write_bytes(b"x" * 10)
    v = np.arange(10.0)
    assert resident.remember(str(p), "X", v)
    assert resident.recall(str(p), "X") is v
    assert resident.recall(str(p), "Y") is None
    # a rewrite (new size / mtime) invalidates
    p.write_bytes(b"y" * 11)
    assert resident.recall(str(p), "X") is None
    # so does replacing the file under the same name (new inode)
    assert resident.remember(str(p), "X", v)
    q = tmp_path / "b.bin"
    q.write_bytes(b"y" * 11)
    st = os.stat(p)
    os.utime(q, ns=(st.st_atime_ns, st.st_mtime_ns))
    os.replace(q, p)
    assert resident.recall(str(p), "X") is None
    resident.forget()


def test_budget_evicts_oldest_and_zero_disables(tmp_path, monkeypatch):
    resident.forget()
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", str(3 * 800))
    paths = []
    for i in range(4):
        p = tmp_path / f"f{i}"
        p.write_bytes(b"z")
        paths.append(str(p))
        assert resident.remember(str(p), "X", np.zeros(100))   # 800 bytes each
    assert resident.recall(paths[0], "X") is None
    assert all(resident.recall(q, "X") is not None for q in paths[1:])
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", "0")
    assert not resident.remember(paths[1], "X", np.zeros(100))
    assert resident.recall(paths[1], "X") is None
    resident.forget()


def test_anndata_mirrors_count_their_matrix_and_attached_device_csr(tmp_path, monkeypatch):
    """A remembered TPM AnnData counts X (sparse: data + indices + indptr) against the
    budget, and so does the device CSR consensus attaches to it afterwards: the next
    remember recounts and evicts it."""
    import scipy.sparse as sp

    from cnmf_torch_amd.utils.anndata_lite import AnnData

    resident.forget()
    X = sp.random(50, 40, density=0.2, format="csr", random_state=0, dtype=np.float32)
    a = AnnData(X=X)
    xb = X.data.nbytes + X.indices.nbytes + X.indptr.nbytes
    assert resident._nbytes(a) == xb
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", str(2 * xb + 100))
    p, q = tmp_path / "tpm", tmp_path / "other"
    p.write_bytes(b"a")
    q.write_bytes(b"b")
    assert resident.remember(str(p), "adata", a)
    # consensus attaches an (emulated) device CSR of the same size
    a.__dict__["_cnmf_device_csr"] = {("cuda:0", id(X)): X.copy()}
    assert resident._nbytes(a) == 2 * xb
    assert resident.remember(str(q), "X", np.zeros(xb // 8 + 1))   # no longer fits beside it
    assert resident.recall(str(p), "adata") is None
    resident.forget()

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

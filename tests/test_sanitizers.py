"""Host-code sanitizers: the native HDF5 layer built with
AddressSanitizer + UBSan and driven through an embedding executable that links the
sanitizer runtimes (tools/asan_h5io.sh).  GPU sanitizers are not used on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/conda/lib/libhdf5.so"),
                    reason="needs g++ and libhdf5")
def test_h5io_asan_ubsan_roundtrip(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_h5io.sh")], env=env,
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "h5io sanitizer round trip: OK" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out

# Round trips through the sanitized _h5io module: dense/CSR matrices, strings, bools,
# categoricals, attributes, partial row reads, missing paths (error paths included).
import os
import tempfile

import numpy as np
import _h5io

d = tempfile.mkdtemp()
fn = os.path.join(d, "t.h5")
rs = np.random.default_rng(0)
f = _h5io.File(fn, "w")
f.create_group("/g")
for dt in (np.float32, np.float64, np.int32, np.int64, np.int8):
    a = (rs.random((37, 5)) * 100).astype(dt)
    f.write_array(f"/g/a_{np.dtype(dt).name}", a, 4)
f.write_strings("/g/s", ["alpha", "", "gamma" * 50, "δ-utf8"])
f.write_strings("/g/empty", [])
f.write_array("/g/b", np.array([True, False, True]), 0)
f.set_attr("/g", "encoding-type", "dataframe")
f.set_attr("/g", "column-order", ["a", "b"])
del f
f = _h5io.File(fn, "r")
for dt in (np.float32, np.float64, np.int32, np.int64, np.int8):
    x = f.read(f"/g/a_{np.dtype(dt).name}", 0, -1)
    assert x.shape == (37, 5), x.shape
    part = f.read(f"/g/a_{np.dtype(dt).name}", 3, 11)
    assert part.shape == (8, 5)
assert list(f.read("/g/s", 0, -1)) == ["alpha", "", "gamma" * 50, "δ-utf8"]
assert len(f.read("/g/empty", 0, -1)) == 0
assert list(f.read("/g/b", 0, -1)) == [True, False, True]
attrs = f.attrs("/g")
assert attrs["encoding-type"] == "dataframe"
assert f.exists("/g/s") and not f.exists("/nope")
try:
    f.read("/nope", 0, -1)
    raise SystemExit("missing path did not raise")
except Exception as e:  # _h5io.H5Error
    assert "nope" in str(e)
print("h5io sanitizer round trip: OK")

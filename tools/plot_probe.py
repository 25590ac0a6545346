"""Clustergram render time in this process (the figure child's job at the e2e shape:
900 spectra): matplotlib import, first and second render, and the PNG encode share.
One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MPLBACKEND", "Agg")
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


def main() -> int:
    t0 = time.perf_counter()
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot  # noqa: F401
    t_imp = time.perf_counter() - t0
    from scipy.spatial.distance import cdist

    from cnmf_torch_amd.utils import plotting

    rng = np.random.default_rng(0)
    n = 900
    X = rng.random((n, 20))
    D = cdist(X, X)
    labels = pd.Series(rng.integers(1, 10, n), index=[f"s{i}" for i in range(n)])
    dens = pd.DataFrame(rng.random(n) * 0.3, columns=["local_density"])
    enc = []
    orig = plotting.write_png_rgba

    def timed(*a, **kw):
        t = time.perf_counter()
        orig(*a, **kw)
        enc.append(time.perf_counter() - t)

    plotting.write_png_rgba = timed
    out = {"import_s": round(t_imp, 3)}
    for rep in range(3):
        t = time.perf_counter()
        plotting.clustergram(D, labels, dens, np.ones(n, bool), 0.1, "/tmp/cg_probe.png",
                             close=True)
        out[f"render{rep}_s"] = round(time.perf_counter() - t, 3)
        out[f"encode{rep}_s"] = round(enc[-1], 3)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Child process of plotting.PlotWorker: import matplotlib at once (overlapping the
parent's GPU work), then draw every job read from stdin, acknowledge each on stdout
("ok <id>" / "err <id>"), and exit at EOF."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import matplotlib  # noqa: E402

matplotlib.use("Agg")
import matplotlib.pyplot  # noqa: E402,F401
# the Agg canvas module loads lazily at a process's first figure (~0.3 s): now, while the
# parent computes, instead of inside the first job
import matplotlib.backends.backend_agg  # noqa: E402,F401
import numpy as np  # noqa: E402
# the clustergram's leaf order (average linkage), loaded before the first job too
import scipy.cluster.hierarchy  # noqa: E402,F401
import scipy.spatial.distance  # noqa: E402,F401

import plotting  # noqa: E402  (this directory: numpy / matplotlib only -- no pandas)


def main() -> int:
    for line in sys.stdin:
        if not line.strip():
            continue
        job = json.loads(line)
        try:
            with np.load(job["npz"], allow_pickle=False) as f:
                arrays = {k: f[k] for k in f.files}
            plotting.draw_job(job["kind"], job["path"], arrays)
            print(f"ok {job['id']}", flush=True)
        except Exception:
            print(f"err {job['id']}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

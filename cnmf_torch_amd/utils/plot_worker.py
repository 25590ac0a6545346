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

import plotting  # noqa: E402  (this directory: numpy / pandas / matplotlib only)


def _warm() -> None:
    """A throwaway figure with the artists the jobs use (text, ticks, image, histogram,
    colour bar, grid spec), drawn while the parent still computes: a process's first
    draw loads the fonts and fills the renderer's caches, which would otherwise land on
    the first real figure, and the figures are the pipeline's last wait."""
    import io

    import matplotlib.pyplot as plt

    fig, (a0, a1) = plt.subplots(1, 2, figsize=(3, 2))
    im = a0.imshow(np.arange(16.0).reshape(4, 4), interpolation="none", aspect="auto",
                   rasterized=True)
    a1.hist(np.arange(10.0), bins=np.linspace(0, 10, 5))
    a1.plot([0, 1], [1, 0], "o-")
    a1.set_title("Stability")
    a1.set_xlabel("Number of Components\n(k)")
    a1.axvline(1.0, linestyle="--", color="k")
    fig.colorbar(im, ax=a0, orientation="horizontal")
    fig.savefig(io.BytesIO(), format="png", dpi=250)
    plt.close(fig)


def main() -> int:
    try:
        _warm()
    except Exception:
        pass
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

"""Probe: Harmony-sized device k-means (cells x PCs: 500k x 20, k = 100, 10 restarts,
25 Lloyd iterations): wall time of k-means++ and of Lloyd separately."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnmf_torch_amd.models import consensus as C  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500000
    rs = np.random.default_rng(0)
    centers = rs.normal(size=(60, 20)) * 3
    X = torch.from_numpy(centers[rs.integers(0, 60, n)] + rs.normal(size=(n, 20))).cuda()
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = torch.Generator().manual_seed(rep)
        c0 = C._kmeanspp_batched(X, 100, g, 10)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        lab, inertia = C._lloyd_batched(X, c0, 25, 1e-9)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"n={n}: kmeans++ {1e3 * (t1 - t0):.1f} ms, Lloyd {1e3 * (t2 - t1):.1f} ms",
              flush=True)


if __name__ == "__main__":
    main()

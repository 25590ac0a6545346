"""Five fused Lloyd steps (ops.kmeans_step, kmeans.hip) at Harmony's init shape -- 500k
cells x 50 PCs, 100 centroids, 10 restarts -- for PMC counter passes of that kernel alone.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python tools/kmeans_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cnmf_torch_amd import ops  # noqa: E402


def main():
    n, d, k, r = 500000, 50, 100, 10
    g = torch.Generator().manual_seed(0)
    X = torch.randn((n, d), generator=g, dtype=torch.float64).cuda()
    C = torch.randn((r, k, d), generator=g, dtype=torch.float64).cuda()
    ops.kmeans_step(X, C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        ops.kmeans_step(X, C)
    torch.cuda.synchronize()
    print(f"kmeans_step: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per call")


if __name__ == "__main__":
    main()

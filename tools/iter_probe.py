"""Probe: inner-solve iteration counts of the headline bench config (bench.py): mean
online passes, H / W inner iterations per solve call, per replicate."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=K, seed=0)).cuda()
    opts = NMFOptions(n_components=K, init="random", beta_loss="frobenius", algo="mu",
                      mode="online", tol=1e-4, online_chunk_size=5000,
                      online_chunk_max_iter=1000)
    solver = NMFBatchSolver(X, opts)
    rs = np.random.RandomState(14)
    for rep in range(2):
        res = solver.run([int(s) for s in rs.randint(1, 2 ** 31 - 1, 100)])
        passes = np.asarray(res.n_iter, dtype=np.float64)
        hi = np.asarray(res.stats["h_inner_iters"], dtype=np.float64)
        wi = np.asarray(res.stats["w_inner_iters"], dtype=np.float64)
        nch = -(-X.shape[0] // 5000)
        print(f"K={K} run {rep}: passes mean {passes.mean():.2f} max {passes.max():.0f}; "
              f"H iters/solve {hi.sum() / (passes.sum() * nch):.1f} "
              f"(max rep {hi.max() / passes[hi.argmax()] / nch:.1f}); "
              f"W iters/solve {wi.sum() / (passes.sum() * nch):.1f}", flush=True)
        h = np.bincount(passes.astype(np.int64))
        print("  replicates per pass count: " +
              ", ".join(f"{p}:{c}" for p, c in enumerate(h) if c), flush=True)


if __name__ == "__main__":
    main()

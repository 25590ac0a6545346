"""Host-side cProfile of bench.py steps (GPU asynchronous): which host calls the step
spends its wall time in -- launch enqueue, synchronisation, pinned copies.
usage: python tools/step_cprofile.py [frobenius|kullback-leibler] [steps]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix  # noqa: E402


def main():
    loss = sys.argv[1] if len(sys.argv) > 1 else "frobenius"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).cuda()
    s = NMFBatchSolver(X, NMFOptions(n_components=10, beta_loss=loss,
                                     online_chunk_max_iter=1000))
    rs = np.random.RandomState(14)

    def step():
        r = s.run_concurrent([int(v) for v in rs.randint(1, 2 ** 31 - 1, 100)], n_streams=1)
        r.W.cpu()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"{loss}: {1e3 * (time.perf_counter() - t0) / steps:.2f} ms per step (profiled)")
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(25)
    print(out.getvalue())


if __name__ == "__main__":
    main()

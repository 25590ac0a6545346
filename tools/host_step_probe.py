"""Host time of the headline's solver.run per batch: cProfile of ``--steps`` warm
100-replicate K = 10 batches (bench.py's default shape), with the GPU idle time between
batches from CUDA events around each run -- where the ~0.6 ms per step outside the pass
loop goes (tools/gap_summary.py shows it as idle gaps before the first kernels of a run).

    python tools/host_step_probe.py [--steps 20] [--out gpurun_out/host_step.txt]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).cuda()
    opts = NMFOptions(n_components=10, init="random", tol=1e-4, online_chunk_size=5000,
                      online_chunk_max_iter=1000)
    solver = NMFBatchSolver(X, opts)
    np.random.seed(14)
    seeds = np.random.randint(1, 2 ** 31 - 1, size=100 * (a.steps + a.warmup))
    for i in range(a.warmup):
        solver.run_concurrent([int(s) for s in seeds[i * 100:(i + 1) * 100]], n_streams=1)
    torch.cuda.synchronize()
    # host wall per call of the run's setup / teardown pieces (no profiler overhead)
    import collections
    import functools

    from cnmf_torch_amd.models import nmf as nmf_mod
    from cnmf_torch_amd.models import nmf_batch

    acc = collections.defaultdict(lambda: [0, 0.0])

    def timed(owner, name, label):
        fn = getattr(owner, name)

        @functools.wraps(fn)
        def w(*args, **kw):
            t = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                acc[label][0] += 1
                acc[label][1] += time.perf_counter() - t
        setattr(owner, name, w)

    for owner, name in ((nmf_mod, "init_into"), (nmf_mod.NMFBatchSolver, "_init_err_frob"),
                        (nmf_mod.NMFBatchSolver, "_fused_ok"), (nmf_mod.NMFBatchSolver, "_steps"),
                        (nmf_mod.NMFBatchSolver, "_arena"), (nmf_mod.NMFBatchSolver, "_online_frob"),
                        (nmf_mod.NMFBatchSolver, "run"), (nmf_batch._Batch, "__init__"),
                        (nmf_batch._Batch, "finalize"), (nmf_mod.NMFBatchSolver, "stats_gemm"),
                        (nmf_mod.NMFBatchSolver, "_enqueue_fused")):
        timed(owner, name, f"{getattr(owner, '__name__', owner)}.{name}")
    for i in range(a.warmup, a.warmup + a.steps):
        solver.run_concurrent([int(v) for v in seeds[i * 100:(i + 1) * 100]], n_streams=1)
    torch.cuda.synchronize()
    lines = [f"{k:60s} {v[0] / a.steps:6.1f} calls/run {1e6 * v[1] / a.steps:9.1f} us/run"
             for k, v in sorted(acc.items(), key=lambda kv: -kv[1][1])]
    print("\n".join(lines))
    pr = cProfile.Profile()
    walls = []
    t0 = time.perf_counter()
    pr.enable()
    for i in range(a.warmup, a.warmup + a.steps):
        s = time.perf_counter()
        solver.run_concurrent([int(v) for v in seeds[i * 100:(i + 1) * 100]], n_streams=1)
        walls.append(time.perf_counter() - s)
    pr.disable()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
    text = ("\n".join(lines) + "\n\n" +
            f"steps {a.steps}: {1e3 * total / a.steps:.3f} ms per run (cProfile on), "
            f"run wall median {1e3 * float(np.median(walls)):.3f} ms\n" + buf.getvalue())
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(text)
    print(text[:6000])


if __name__ == "__main__":
    main()

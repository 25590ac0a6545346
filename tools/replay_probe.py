"""Probe: run_concurrent (two streams) vs the same groups run serially, repeated with
fresh solvers -- which group differs, and is it reproducible (test_run_concurrent_*)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnmf_torch_amd import ops  # noqa: E402
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402

rs = np.random.default_rng(5)
N, G, K = 4000, 600, 9
X = torch.from_numpy((rs.gamma(1, 1, (N, K)) @ rs.gamma(0.5, 1, (K, G)) +
                      0.1 * rs.random((N, G))).astype(np.float32)).cuda()
opts = NMFOptions(n_components=K, online_chunk_size=1500, online_max_pass=6)
seeds = list(range(100, 132))
ref = None
for trial in range(int(os.environ.get('TRIALS', '3'))):
    solver = NMFBatchSolver(X, opts)
    both = solver.run_concurrent(seeds, n_streams=2)
    with ops.coop_share(2):
        a = solver.run(seeds[:16])
        b = solver.run(seeds[16:])
        fa = NMFBatchSolver(X, opts).run(seeds[:16])
        fb = NMFBatchSolver(X, opts).run(seeds[16:])
    ser = torch.cat([a.W, b.W])
    fr = torch.cat([fa.W, fb.W])
    if ref is None:
        ref = ser.clone()
    d = lambda u, v: [(u[:144] - v[:144]).abs().max().item(), (u[144:] - v[144:]).abs().max().item()]
    print(f"trial {trial}: both-vs-serial {d(both.W, ser)} fresh-vs-serial {d(fr, ser)} "
          f"serial-vs-trial0 {d(ser, ref)} passes a {a.n_iter.tolist()} b {b.n_iter.tolist()} "
          f"both {both.n_iter.tolist()}", flush=True)

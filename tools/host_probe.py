"""Probe: host enqueue time vs GPU wait per online pass of the bench shape
(NMFBatchSolver(profile=True) records both; 3 runs of 100 replicates).  The output is
profiles/r1_host_probe_v25.log."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, collections
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix
X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).cuda()
s = NMFBatchSolver(X, NMFOptions(n_components=10), profile=True)
for i in range(3):
    s.timings.clear()
    r = s.run(list(range(1 + 100 * i, 101 + 100 * i)))
h = s.timings["host_pass"]; w = s.timings["wait_pass"]
print("passes", len(h), "host total ms", sum(t for _, t in h) * 1e3, "wait total ms", sum(t for _, t in w) * 1e3)
for (n, t), (_, tw) in zip(h, w):
    print(f"n={n:3d} host {t*1e6:7.0f} us  wait/compact {tw*1e6:7.0f} us")

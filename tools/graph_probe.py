"""Probe: eager pass enqueue vs HIP-graph replay (CNMF_GRAPHS) on the bench shape.
Prints per-run wall time of 100 replicates for both modes, the eager host-enqueue /
GPU-wait split per pass, and the capture cost of one pass graph."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnmf_torch_amd.models import nmf  # noqa: E402
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix  # noqa: E402

X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).cuda()
for mode in ("0", "1", "0"):
    os.environ["CNMF_GRAPHS"] = mode
    s = NMFBatchSolver(X, NMFOptions(n_components=10), profile=True)
    walls = []
    for i in range(6):
        s.timings.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.run(list(range(1 + 100 * i, 101 + 100 * i)))
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    h = s.timings.get("host_pass", [])
    w = s.timings.get("wait_pass", [])
    print(f"CNMF_GRAPHS={mode}: run ms", [round(x * 1e3, 2) for x in walls], flush=True)
    print(f"   last run: eager passes {len(h)}, host enqueue ms {sum(t for _, t in h)*1e3:.2f}, "
          f"wait ms {sum(t for _, t in w)*1e3:.2f}", flush=True)
    for (n, t), (_, tw) in list(zip(h, w))[:12]:
        print(f"   n={n:3d} host {t*1e6:7.0f} us  wait/compact {tw*1e6:7.0f} us", flush=True)
# cost of capturing one pass-sized kernel sequence
g = torch.cuda.CUDAGraph()
a = torch.randn(1 << 20, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.graph(g):
    for _ in range(40):
        a.mul_(1.0001)
torch.cuda.synchronize()
t1 = time.perf_counter()
g.replay()
torch.cuda.synchronize()
t2 = time.perf_counter()
g.replay()
torch.cuda.synchronize()
t3 = time.perf_counter()
print(f"40-kernel graph: capture+instantiate {1e3*(t1-t0):.2f} ms, first replay "
      f"{1e3*(t2-t1):.2f} ms, replay {1e3*(t3-t2):.3f} ms")

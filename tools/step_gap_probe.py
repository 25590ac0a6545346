"""Probe: where the host time between bench steps goes (the GPU idles ~0.3 ms per 7.6 ms
step; profiles/r3aj_kernel_stats_cf0.5.txt).  Runs the headline shape (100 replicates,
10k x 2k, K=10) for a few warmup steps, then profiles two steps with torch.profiler
(CPU ops + stacks) and prints (1) the host wall of each phase of NMFBatchSolver.run,
(2) the CPU ops that issue copies, with their Python call sites."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

dev = torch.device("cuda", 0)
X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).to(dev)
opts = NMFOptions(n_components=10, init="random", beta_loss="frobenius", algo="mu",
                  mode="online", tol=1e-4, online_chunk_size=5000, online_chunk_max_iter=1000)
s = NMFBatchSolver(X, opts)
rng = np.random.RandomState(14)
cs = torch.cuda.Stream(dev)
buf = torch.empty((1000, 2000), dtype=torch.float32, pin_memory=True)


def step():
    r = s.run([int(v) for v in rng.randint(1, 2 ** 31 - 1, size=100)])
    cs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cs):
        buf.copy_(r.W, non_blocking=True)
    r.W.record_stream(cs)
    return r


for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step()
torch.cuda.synchronize()
print(f"plain: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step")

import collections, traceback
sites = collections.Counter()
def _wrap(name):
    orig = getattr(torch.Tensor, name)
    def f(self, *a, **k):
        if self.is_cuda:
            st = traceback.extract_stack(limit=5)[:-1]
            sites[(name,) + tuple(f"{os.path.basename(fr.filename)}:{fr.lineno}:{fr.name}" for fr in st)] += 1
        return orig(self, *a, **k)
    setattr(torch.Tensor, name, f)
for nm in ("item", "__bool__", "__int__", "__float__", "__index__", "tolist", "cpu", "numpy"):
    _wrap(nm)
for _ in range(2):
    step()
torch.cuda.synchronize()
print("device->host syncs per step (2 steps):")
for k, v in sites.most_common(40):
    print(f"{v / 2:6.1f}  {k[0]:10s} " + "  <-  ".join(reversed(k[1:])))

from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
    for _ in range(2):
        step()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ka if any(k in e.key for k in ("copy", "_to_copy", "item", "nonzero",
                                                  "local_scalar", "synchronize", "pin"))]
rows.sort(key=lambda e: -e.cpu_time_total)
for e in rows[:30]:
    print(f"{e.key:32s} n={e.count:4d} cpu_total={e.cpu_time_total / 2:9.1f} us/step")
    for fr in (e.stack or [])[:6]:
        print("      ", fr)
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))

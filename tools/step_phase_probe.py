import os, sys, time
sys.path.insert(0, "/root/repo")
os.chdir("/root/repo")
import numpy as np, torch
from cnmf_torch_amd.models import nmf as M
from cnmf_torch_amd import ops
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix
X = torch.from_numpy(normalized_counts_matrix(10000, 2000, n_programs=10, seed=0)).cuda()
s = M.NMFBatchSolver(X, M.NMFOptions(n_components=10))
rs = np.random.RandomState(14)
T = {}
def tm(name, f):
    t = time.perf_counter(); r = f(); T.setdefault(name, []).append(time.perf_counter() - t); return r
orig_fin = M._Batch.finalize
M._Batch.finalize = lambda self: tm("finalize", lambda: orig_fin(self))
orig_cc = ops.coop_check
ops.coop_check = lambda d=None: tm("coop_check", lambda: orig_cc(d))
orig_online = M.NMFBatchSolver._online_frob
M.NMFBatchSolver._online_frob = lambda self, st: tm("online_frob", lambda: orig_online(self, st))
for i in range(12):
    seeds = [int(v) for v in rs.randint(1, 2**31 - 1, 100)]
    t0 = time.perf_counter()
    r = tm("run", lambda: s.run(seeds))
    tm("W.cpu", lambda: r.W.cpu())
    T.setdefault("step", []).append(time.perf_counter() - t0)
for k, v in T.items():
    print(f"{k:12s} median {1e3*np.median(v[2:]):7.3f} ms")

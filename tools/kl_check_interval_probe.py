"""CPU probe: online KL with the usage block objective checked every 10/5/3/2 steps --
passes, convergence, final KL vs batch MU, usage/spectra iterations (4000 x 2000, K=10,
2 chunks, 4 seeds).  Output: profiles/r2_kl_check_interval_probe.log."""
import sys, time, numpy as np, torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnmf_torch_amd.models import nmf as M
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix
torch.set_num_threads(8)
N = 4000
X = torch.from_numpy(normalized_counts_matrix(N, 2000, n_programs=10, seed=0))
seeds = [1, 2, 3, 4]
b = M.NMFBatchSolver(X, M.NMFOptions(n_components=10, beta_loss="kullback-leibler", mode="batch", batch_max_iter=500)).run(seeds)
print("batch err", b.err.round(2), "iters", b.n_iter, flush=True)
for ce in [10, 5, 3, 2]:
    for wt in [5e-3]:
        t = time.time()
        o = M.NMFOptions(n_components=10, beta_loss="kullback-leibler", online_chunk_size=N//2, online_chunk_max_iter=1000, inner_check_every=ce, online_beta_w_tol=wt)
        s = M.NMFBatchSolver(X, o)
        r = s.run(seeds)
        print(f"ce={ce} wtol={wt}: passes {r.n_iter} conv {r.converged} err {r.err.round(2)} rel-to-batch {(r.err/b.err-1).round(4)} h_it {np.asarray(r.stats['h_inner_iters'])} w_it {np.asarray(r.stats['w_inner_iters'])} {time.time()-t:.1f}s", flush=True)

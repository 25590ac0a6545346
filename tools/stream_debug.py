"""Trace a small streaming run's batch layout pass by pass (debug aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cnmf_torch_amd.models import nmf
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=10, seed=6)).cuda()
opts = nmf.NMFOptions(n_components=10, online_chunk_size=2000, online_chunk_max_iter=1000)
solver = nmf.NMFBatchSolver(X, opts)
orig_loop = solver._stream_loop
orig_pass = solver._fused_pass


def traced_pass(st, steps, fb, final=False):
    print("pass: n_act", st.n_act, "groups", [(g.K, g.p0, g.n) for g in st.groups],
          "fb rows", fb["B"].shape, flush=True)
    return orig_pass(st, steps, fb, final)


def traced_loop(st, steps, cur):
    print("loop start: n_act", st.n_act, "groups", st.groups, flush=True)
    return orig_loop(st, steps, cur)


orig_stock = solver._stream_stock


def traced_stock(st, K, cur):
    f = st.feed
    r = f.rings.get(K)
    print("stock K", K, "queue", len(f.queue.get(K, [])), "known_head", f.known_head.get(K),
          "published", None if r is None else r["published"], "done", f.done,
          "ctr", f.ctr.tolist(), flush=True)
    return orig_stock(st, K, cur)


solver._stream_stock = traced_stock
solver._fused_pass = traced_pass
solver._stream_loop = traced_loop
res = solver.run_stream(list(range(101, 131)), live=8)
print("passes", res.n_iter.tolist(), "err", np.round(res.err, 4).tolist()[:5], res.stats)

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cnmf_torch_amd import ops
from cnmf_torch_amd.ops import reference
dev = torch.device("cuda")
for K, n in ((1, 10), (3, 7), (3, 3001), (10, 5000)):
    R = 2
    x = torch.rand((R, K, n), device=dev) + 0.5
    numer = torch.rand((R, K, n), device=dev) + 0.5
    W = torch.rand((R, K, 8), device=dev)
    gram = torch.bmm(W, W.transpose(1, 2))
    xr = x.cpu().double().clone()
    xg = x.clone()
    ops.solve("mu", xg, numer, gram, max_iter=1, tol=-1.0)
    reference.solve(0, xr, numer.cpu().double(), gram.cpu().double(), None, 1, -1.0, 0, 0, 0, 1e-16, None, None, None)
    torch.cuda.synchronize()
    d = (xg.cpu().double() - xr).abs().max().item()
    print(K, n, "maxdiff", d, "gpu", xg[0, 0, :4].tolist(), "ref", xr[0, 0, :4].tolist(), flush=True)

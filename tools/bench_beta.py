"""Micro-benchmark of the fused beta-MU contraction (beta_mu.hip) vs the eager
PyTorch sequence it replaces (bmm -> clamp/div -> bmm), on the bench shape."""
import argparse
import json
import time

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cnmf_torch_amd import ops
from cnmf_torch_amd.ops import reference


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=100)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--N", type=int, default=10000)
    ap.add_argument("--G", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    R, K, N, G = a.R, a.K, a.N, a.G
    X = torch.rand((N, G), device=dev)
    HT = torch.rand((R, K, N), device=dev) + 0.1
    W = torch.rand((R, K, G), device=dev) + 0.1
    out = {}
    for side in ("h", "w"):
        t = timeit(lambda: ops.beta_contract(side, X, HT, W, 1.0, 1e-10))
        flops = 4.0 * R * K * N * G
        out[f"fused_{side}_ms"] = t * 1e3
        out[f"fused_{side}_tflops"] = flops / t / 1e12

    def eager_h():  # reference chunked eager math on GPU (what nmf-torch does per replicate)
        for r0 in range(0, R, 10):
            P = torch.bmm(HT[r0:r0 + 10].transpose(1, 2), W[r0:r0 + 10])
            Q = X / P.clamp_min(1e-10)
            torch.bmm(W[r0:r0 + 10], Q.transpose(1, 2))
    t = timeit(eager_h, 2)
    out["eager_h_ms"] = t * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()

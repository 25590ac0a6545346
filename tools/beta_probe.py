"""Probe: time of the fused beta-divergence kernels (csrc/kernels/beta_mu.hip) on the
bench chunk shape (R replicates, K, c cells x G genes): usage update, W-side
contraction and the loss-only pass.  Prints microseconds per call and the fp32-MFMA
bound for the same work (7 16x16x4 MFMAs per 16x16 tile at K <= 12)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnmf_torch_amd import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=100)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--c", type=int, default=5000)
    ap.add_argument("--G", type=int, default=2000)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.poisson(torch.rand(a.c, a.G, device="cuda", generator=g) * 2)
    HT = torch.rand(a.R, a.K, a.c, device="cuda", generator=g) + 0.1
    W = torch.rand(a.R, a.K, a.G, device="cuda", generator=g) + 0.1
    H0 = HT.clone()
    tiles = a.R * ((a.c + 15) // 16) * ((a.G + 15) // 16)
    bound_us = tiles * 7 * 32 / (1024 * 2.4e9) * 1e6
    cases = {
        "update_h": lambda: (HT.copy_(H0), ops.beta_update_h(X, HT, W, 1.0, 1e-16)),
        "contract_w": lambda: ops.beta_contract("w", X, HT, W, 1.0, 1e-16),
        "loss_h": lambda: ops.beta_contract("h", X, HT, W, 1.0, 1e-16, want_num=False,
                                            want_loss=True),
    }
    for name, fn in cases.items():
        if a.only and name != a.only:
            continue
        us = timed(fn)
        print(f"{name:10s} R={a.R} K={a.K} c={a.c} G={a.G}: {us:8.1f} us "
              f"(fp32 MFMA bound {bound_us:.0f} us, {bound_us / us * 100:.0f}%)", flush=True)


if __name__ == "__main__":
    main()

"""Probe: split-bf16 beta kernels (csrc/kernels/beta_planes.hip) on the bench chunk shape:
per-MU-step time of the fused usage block (nsteps per launch), the W-side partials and the
loss-only pass; the first-generation fp32-MFMA kernels (beta_mu.hip) for comparison."""
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
    ap.add_argument("--beta", type=float, default=1.0)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.poisson(torch.rand(a.c, a.G, device="cuda", generator=g) * 2)
    XT = X.t().contiguous()
    HT = torch.rand(a.R, a.K, a.c, device="cuda", generator=g) + 0.1
    W = torch.rand(a.R, a.K, a.G, device="cuda", generator=g) + 0.1
    H0 = HT.clone()
    elems = a.R * a.c * a.G
    pw = ops.beta_panels(W, a.beta)
    ph = ops.beta_panels(HT, a.beta)
    ns = 10
    cases = {
        "h_block10 (per step)": (lambda: (HT.copy_(H0), ops.beta_h_block(
            X, HT, W, a.beta, 1e-16, ns, panels=pw)), ns),
        "w_partials": (lambda: ops.beta_w_partials(X, XT, HT, W, a.beta, 1e-16, panels=ph), 1),
        "loss": (lambda: ops.beta_loss(X, HT, W, a.beta, 1e-16, panels=pw), 1),
        "panels W": (lambda: ops.beta_panels(W, a.beta, out=pw), 1),
        "panels H": (lambda: ops.beta_panels(HT, a.beta, out=ph), 1),
        "old update_h": (lambda: (HT.copy_(H0), ops.beta_update_h(X, HT, W, a.beta, 1e-16)), 1),
        "old contract_w": (lambda: ops.beta_contract("w", X, HT, W, a.beta, 1e-16), 1),
    }
    for name, (fn, div) in cases.items():
        us = timed(fn) / div
        print(f"{name:22s} R={a.R} K={a.K} c={a.c} G={a.G} beta={a.beta}: {us:8.1f} us "
              f"({elems / us / 1e6:.2f} Gelem/ms)", flush=True)


if __name__ == "__main__":
    main()

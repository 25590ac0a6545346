"""Probe: per-iteration cost of the fused inner solve (csrc/kernels/solve_core.h) on the
bench shapes, by variant (streaming / register-resident) and cooperative split S.
Runs a fixed number of MU sweeps (tol < 0: no early stop) and times the launch."""
import argparse
import time

import torch

import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnmf_torch_amd import ops


def case(R, K, n, iters, variant, coop, conv_mode=0, reps=5):
    g = torch.Generator(device="cuda").manual_seed(0)
    W = torch.rand(R, K, 64, device="cuda", generator=g)
    gram = torch.bmm(W, W.transpose(1, 2)).contiguous()
    x0 = torch.rand(R, K, n, device="cuda", generator=g)
    numer = torch.rand(R, K, n, device="cuda", generator=g) * 16
    x = x0.clone()

    def run():
        x.copy_(x0)
        ops.solve("mu", x, numer, gram, max_iter=iters, tol=-1.0, conv_mode=conv_mode,
                  check_every=10, variant=variant, coop=coop)

    run()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(reps):
        ev0.record()
        run()
        ev1.record()
        torch.cuda.synchronize()
        best = min(best, ev0.elapsed_time(ev1) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    K = a.k
    for R, n, label in ((100, 5000, "H-side n=100"), (50, 5000, "H-side n=50"),
                        (100, 2000, "W-side n=100")):
        for variant, coop in (("stream", "auto"), ("stream", 1), ("reg", "auto"),
                              ("mfma", "auto")):
            try:
                t10 = case(R, K, n, 10, variant, coop)
                t40 = case(R, K, n, 40, variant, coop)
                print(f"{label:14s} K={K} {variant:6s} coop={coop!s:4s}: 10 it {t10:7.1f} us, "
                      f"40 it {t40:7.1f} us -> {(t40 - t10) / 30:6.2f} us/iter", flush=True)
            except Exception as e:  # variant not applicable to the shape
                print(f"{label:14s} K={K} {variant:6s} coop={coop!s:4s}: n/a ({e})", flush=True)
        for variant in ("reg", "mfma"):
            try:
                t10 = case(R, K, n, 10, variant, "auto", 1)
                t40 = case(R, K, n, 40, variant, "auto", 1)
                print(f"{label:14s} K={K} {variant:6s} loss-conv : 10 it {t10:7.1f} us, 40 it "
                      f"{t40:7.1f} us -> {(t40 - t10) / 30:6.2f} us/iter", flush=True)
            except Exception as e:
                print(f"{label:14s} K={K} {variant:6s} loss-conv : n/a ({e})", flush=True)


if __name__ == "__main__":
    main()

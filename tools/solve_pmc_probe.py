"""Probe for hardware counters of the fused inner solve: the bench's H-side shape
(100 replicates x K=10 x 5000 cells), 40 MU sweeps with the objective stop, per variant.
Run under rocprofv3 --pmc; the variant is argv[1] (reg | mfma)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnmf_torch_amd import ops  # noqa: E402


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "mfma"
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 10   # 1000: sweeps only
    R, K, n = 100, 10, 5000
    g = torch.Generator(device="cuda").manual_seed(0)
    W = torch.rand(R, K, 64, device="cuda", generator=g)
    gram = torch.bmm(W, W.transpose(1, 2)).contiguous()
    x0 = torch.rand(R, K, n, device="cuda", generator=g)
    numer = torch.rand(R, K, n, device="cuda", generator=g) * 16
    for _ in range(5):
        x = x0.clone()
        ops.solve("mu", x, numer, gram, max_iter=40, tol=-1.0, conv_mode=1,
                  check_every=every, variant=variant, coop="auto")
    torch.cuda.synchronize()
    print("done", variant, flush=True)


if __name__ == "__main__":
    main()

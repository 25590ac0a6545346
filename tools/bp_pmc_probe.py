"""PMC probe of the split-bf16 beta kernels (beta_planes.hip) on the bench chunk shape:
``h`` = 3 launches of a 10-step fused usage block, ``w`` = 3 W-side partial launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnmf_torch_amd import ops  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "h"
    R, K, c, G = 100, 10, 5000, 2000
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.poisson(torch.rand(c, G, device="cuda", generator=g) * 2)
    HT = torch.rand(R, K, c, device="cuda", generator=g) + 0.1
    W = torch.rand(R, K, G, device="cuda", generator=g) + 0.1
    if which == "h":
        pw = ops.beta_panels(W, 1.0)
        for _ in range(3):
            ops.beta_h_block(X, HT, W, 1.0, 1e-16, 10, panels=pw)
    else:
        XT = X.t().contiguous()
        ph = ops.beta_panels(HT, 1.0)
        for _ in range(3):
            ops.beta_w_partials(X, XT, HT, W, 1.0, 1e-16, panels=ph)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

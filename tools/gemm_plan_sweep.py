"""Tile-variant x k-split sweep of the split-plane GEMM (gemm_planes.hip) at the fused
step's main-pass shapes for K = 10 / 20 / 30 (100 replicates, 10k x 2k, 5000-cell chunks),
in raw-slab mode (what the fused step runs: partial products for the solve, no reduction
pass).  Prints one JSON line per shape with the time of every (variant, ksplit) and the
plan ops.gemm_plan picks, to check the plan against wave quantisation (e.g. 320 tiles on
256 CUs).

    python tools/gemm_plan_sweep.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cnmf_torch_amd import ops  # noqa: E402


def _time(fn, reps=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    h = ops._hip
    shapes = []
    # rows = replicates x K; default the fused step's main-pass rows at K = 10 / 20 / 30
    # (100 replicates) -- or the M values given on the command line
    Ms = [int(a) for a in sys.argv[1:]] or [1000, 2000, 3000]
    for M in Ms:
        shapes += [(f"numerator M={M}", M, 5000, 2048), (f"statistics M={M}", M, 2000, 5056)]
    for name, M, N, Kd in shapes:
        A = torch.rand((M, Kd), device=dev, generator=g)
        B = torch.randint(0, 60, (N, Kd), device=dev, generator=g).float()
        Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device=dev)
        Bp = torch.zeros((1, N, Kd), dtype=torch.int16, device=dev)
        ops.split_planes(A, Ap)
        ops.split_planes(B, Bp)
        pa, pb = 2, 1
        slab = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
        plan = ops.gemm_plan(M, N, Kd, pb)
        res = {}
        for v in (0, 1, 2, 3, 4, 5):
            for ks in (1, 2, 4):
                if Kd // ops.planes_bk(pb) < ks:
                    continue

                def run(v=v, ks=ks):
                    h.gemm_planes(Ap.data_ptr(), Ap.stride(1), Ap.stride(0), M, Bp.data_ptr(),
                                  Bp.stride(1), Bp.stride(0), N, slab.data_ptr(), N, 0, M, N,
                                  Kd, pa, pb, 0, v, ks, slab.data_ptr(), ops.gemm_stages(v),
                                  ops.gemm_kstep(v), 1, 0, ops._stream_ptr(slab))
                try:
                    res[f"v{v}k{ks}"] = round(_time(run), 1)
                except Exception as e:      # a variant the shape / LDS does not allow
                    res[f"v{v}k{ks}"] = str(e)[:40]
        best = min((t, k) for k, t in res.items() if isinstance(t, float))
        print(json.dumps({"shape": name, "M": M, "N": N, "Kd": Kd,
                          "plan": f"v{plan[0]}k{plan[1]}", "plan_us": res.get(f"v{plan[0]}k{plan[1]}"),
                          "best": best[1], "best_us": best[0], "us": res}), flush=True)


if __name__ == "__main__":
    main()

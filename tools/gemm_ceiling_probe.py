"""Ceiling probe for the split-plane GEMMs: the library bf16 GEMM
(hipBLASLt through torch.matmul) on the same work as each main-pass plane GEMM of the
headline bench, timed beside gemm_planes itself.

A plane GEMM with PA A-planes and PB B-planes computes sum_{i + j <= 2} A_i B_j^T: for the
count data of the bench (PA = 2, PB = 1) that is two bf16 products of M x N x Kd, the same
MFMA work as ONE bf16 GEMM with a 2 Kd-deep reduction -- which is what the library is timed
on.  Probe only: the engine keeps gemm_planes (fused slab epilogue, exact planes).

    python tools/gemm_ceiling_probe.py            # prints one JSON line per shape
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cnmf_torch_amd import ops  # noqa: E402


def _time(fn, reps=50, warm=5):
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
    shapes = [("numerator K=10", 1000, 5000, 2048), ("statistics K=10", 1000, 2000, 5056),
              ("numerator K=20", 2000, 5000, 2048), ("statistics K=20", 2000, 2000, 5056)]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, Kd in shapes:
        A = torch.rand((M, Kd), device=dev, generator=g)
        B = torch.randint(0, 60, (N, Kd), device=dev, generator=g).float()
        Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device=dev)
        Bp = torch.zeros((1, N, Kd), dtype=torch.int16, device=dev)
        ops.split_planes(A, Ap)
        ops.split_planes(B, Bp)
        C = torch.empty((M, N), device=dev)
        t_planes = _time(lambda: ops.gemm_planes(C, Ap[:2], Bp, M, N, Kd))
        # the library on the same MFMA work: one bf16 GEMM, 2 Kd deep, fp32 output
        Al = torch.rand((M, 2 * Kd), device=dev, generator=g).to(torch.bfloat16)
        Bl = torch.rand((2 * Kd, N), device=dev, generator=g).to(torch.bfloat16)
        t_lib = _time(lambda: torch.matmul(Al, Bl))
        flops = 2.0 * M * N * 2 * Kd
        print(json.dumps({"shape": name, "M": M, "N": N, "Kd": Kd, "planes": "2A x 1B",
                          "gemm_planes_us": round(t_planes, 2), "hipblaslt_bf16_us": round(t_lib, 2),
                          "planes_vs_library": round(t_lib / t_planes, 3),
                          "planes_tflops": round(flops / t_planes / 1e6, 1),
                          "library_tflops": round(flops / t_lib / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

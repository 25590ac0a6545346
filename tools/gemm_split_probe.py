"""Probe: fp32 GEMM (hipBLASLt fp32 MFMA) vs fp32-accurate bf16 split GEMMs (one bf16
MFMA GEMM over a K-concatenated [hi|mid|lo] operand, fp32 accumulate) on the bench shapes.
Prints time per GEMM and the error against a float64 product."""
import time

import torch

dev = torch.device("cuda")
torch.manual_seed(0)


def split3(x):
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    return h, m, lo


def cat_a(p, terms):
    return torch.cat([p[i] for i, _ in terms], dim=1)


def cat_b(p, terms):
    return torch.cat([p[j] for _, j in terms], dim=1)


T6 = [(0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)]
T3 = [(0, 0), (0, 1), (1, 0)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def run(M, N, Kd, label):
    # A: (M x Kd) like W (spectra), B: (N x Kd) like a chunk of X; C = A B^T
    A = torch.rand(M, Kd, device=dev) * 0.1
    B = torch.poisson(torch.rand(N, Kd, device=dev) * 2) / 1.7
    ref = (A.double() @ B.double().t())
    scale = (A.double().abs() @ B.double().abs().t())
    res = {}
    res["fp32"] = (timeit(lambda: torch.mm(A, B.t())), torch.mm(A, B.t()))
    Bt32 = B.t().contiguous()
    res["fp32_KN"] = (timeit(lambda: torch.mm(A, Bt32)), torch.mm(A, Bt32))
    pa, pb = split3(A), split3(B)
    for name, T in (("bf16x6", T6), ("bf16x3", T3)):
        Ac, Bc = cat_a(pa, T).contiguous(), cat_b(pb, T).contiguous()
        res[name] = (timeit(lambda: torch.mm(Ac, Bc.t(), out_dtype=torch.float32)),
                     torch.mm(Ac, Bc.t(), out_dtype=torch.float32))
        Bt = Bc.t().contiguous()
        res[name + "_KN"] = (timeit(lambda: torch.mm(Ac, Bt, out_dtype=torch.float32)),
                             torch.mm(Ac, Bt, out_dtype=torch.float32))
    split_us = timeit(lambda: cat_a(split3(A), T6))
    flops = 2.0 * M * N * Kd
    for k, (us, C) in res.items():
        err = ((C.double() - ref).abs() / scale.clamp_min(1e-30))
        print(f"{label:28s} {k:10s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF(fp32-eq)  "
              f"err max {err.max().item():.2e} mean {err.mean().item():.2e}", flush=True)
    print(f"{label:28s} split+cat of A (torch eager): {split_us:.1f} us", flush=True)


if __name__ == "__main__":
    run(1000, 5000, 2000, "numer W.Xc^T 1000x5000x2000")
    run(1000, 2000, 5000, "B=HT_c.X_c 1000x2000x5000")
    run(1000, 10000, 2000, "batch W.X^T 1000x10000x2000")

"""Probe: hipBLASLt fp32 time of the two per-chunk GEMMs of the online pass in every
operand / output orientation (the solve kernels could read a transposed numerator).
    numerT (nK x c) = W (nK x G) . X_c^T      or  numer (c x nK) = X_c . W^T
    B      (nK x G) = HT_c (nK x c) . X_c     or  B^T (G x nK)   = X_c^T . HT_c^T
"""
import time

import torch

dev = torch.device("cuda")


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    for nK in (1000, 620, 250):
        N, c, G = 10000, 5000, 2000
        X = torch.rand(N, G, device=dev)
        xc = X[:c]
        W = torch.rand(nK, G, device=dev)
        HT = torch.rand(nK, N, device=dev)
        hc = HT[:, :c]
        hcT = torch.rand(N, nK, device=dev)[:c]     # usages stored cells-major
        o1 = torch.empty(nK, c, device=dev)
        o2 = torch.empty(c, nK, device=dev)
        o3 = torch.empty(nK, G, device=dev)
        o4 = torch.empty(G, nK, device=dev)
        fl = 2.0 * nK * c * G / 1e6
        res = {
            "numerT = W.Xc^T": timeit(lambda: torch.mm(W, xc.t(), out=o1)),
            "numer  = Xc.W^T": timeit(lambda: torch.mm(xc, W.t(), out=o2)),
            "B      = HTc.Xc": timeit(lambda: torch.mm(hc, xc, out=o3)),
            "B^T    = Xc^T.HTc^T": timeit(lambda: torch.mm(xc.t(), hc.t(), out=o4)),
            "B      = Hc^T.Xc (H cells-major)": timeit(lambda: torch.mm(hcT.t(), xc, out=o3)),
            "B^T    = Xc^T.Hc (H cells-major)": timeit(lambda: torch.mm(xc.t(), hcT, out=o4)),
        }
        for k, us in res.items():
            print(f"nK={nK:5d} {k:34s} {us:7.1f} us  {fl / us:6.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()

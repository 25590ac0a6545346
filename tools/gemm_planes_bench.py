"""Split-precision MFMA GEMM (ops.gemm_planes) vs the fp32 library GEMM (torch.mm ->
hipBLASLt) on the shapes of the online NMF step.  fp32-equivalent TFLOP/s (2*M*N*K).

    python tools/gemm_planes_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cnmf_torch_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    shapes = [("numer K=10x100", 1000, 5000, 2000), ("stats K=10x100", 1000, 2000, 5000),
              ("numer grid K=5..13x100", 8100, 5000, 2000), ("stats grid", 8100, 2000, 5000),
              ("numer tail", 80, 5000, 2000), ("stats tail", 80, 2000, 5000)]
    out = []
    for name, M, N, K in shapes:
        A = torch.rand((M, K), device="cuda")
        Bf = torch.randint(0, 50, (N, K), device="cuda").float()
        C = torch.empty((M, N), device="cuda")
        t_lib = timeit(lambda: torch.mm(A, Bf.t(), out=C))
        ref = A.double() @ Bf.double().t()
        lib_err = float((C.double() - ref).abs().max() / ref.abs().max())
        rec = {"shape": name, "M": M, "N": N, "K": K, "fp32_lib_ms": round(t_lib * 1e3, 4),
               "fp32_lib_tflops": round(2 * M * N * K / t_lib / 1e12, 1),
               "fp32_lib_relerr": float(f"{lib_err:.2e}")}
        for pb in (1, 3):
            bk = ops.planes_bk(pb)
            Kd = -(-K // bk) * bk
            Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device="cuda")
            Bp = torch.zeros((pb, N, Kd), dtype=torch.int16, device="cuda")
            ops.split_planes(A, Ap)
            ops.split_planes(Bf, Bp)
            ref = A.double() @ Bf.double().t()
            rec[f"auto_plan_pb{pb}"] = ops.gemm_plan(M, N, Kd, pb)
            variants = [None] + ([(v, k) for v in (0, 1, 2, 3, 4, 5) for k in (1, 2, 4)] if pb == 1
                                 else [])
            for vk in variants:
                if vk is not None:
                    os.environ["CNMF_GEMM_VARIANT"], os.environ["CNMF_GEMM_KSPLIT"] = map(str, vk)
                    ops.refresh_env()
                t = timeit(lambda: ops.gemm_planes(C, Ap, Bp, M, N, Kd))
                ops.gemm_planes(C, Ap, Bp, M, N, Kd)
                err = float((C.double() - ref).abs().max() / ref.abs().max())
                tag = "auto" if vk is None else f"v{vk[0]}k{vk[1]}"
                rec[f"pb{pb}_{tag}"] = [round(t * 1e3, 4), round(2 * M * N * K / t / 1e12, 1),
                                        float(f"{err:.2e}")]
                os.environ.pop("CNMF_GEMM_VARIANT", None)
                os.environ.pop("CNMF_GEMM_KSPLIT", None)
                ops.refresh_env()
            rec["split_A_ms"] = round(timeit(lambda: ops.split_planes(A, Ap)) * 1e3, 4)
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()

"""Large-N benchmarks (BASELINE.json configs 3 and 4) on synthetic data generated on the
device, so host RAM never holds the matrix.

    # config 3: 1M cells x 2k genes, K=10, replicate-parallel (this GPU's share of 200)
    python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 25
    # config 4: 10M cells x 5k genes, K=20, cell-sharded data parallel
    torchrun --nproc-per-node 8 tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --dp
    python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --dp   # whole 200 GB on 1 GPU

With ``--dp`` each rank owns rows [N*r/W, N*(r+1)/W) of X and the solver all-reduces the
[dB | dA] sufficient statistics once per online step over RCCL (NMFBatchSolver with a
DistComm); without it every rank factorises its own replicates of the full matrix.
Data: planted programs (lognormal spectra, Dirichlet usages, Poisson counts), each gene
scaled to unit variance like cNMF's norm_counts; the generator is seeded per row block,
so the matrix is identical for any world size.  Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions  # noqa: E402
from cnmf_torch_amd.parallel.comm import DistComm, LocalComm  # noqa: E402

BLOCK = 1 << 17  # rows per generator block (seeded by block index)


def _programs(G, P, dev, seed=0):
    gs = torch.Generator(device=dev).manual_seed(seed)
    base = torch.empty(G, device=dev).log_normal_(0.0, 1.0, generator=gs)
    S = base.repeat(P, 1)
    nprog = max(1, int(0.15 * G))
    for k in range(P):
        idx = torch.randperm(G, device=dev, generator=gs)[:nprog]
        S[k, idx] *= torch.empty(nprog, device=dev).log_normal_(1.5, 0.5, generator=gs)
    S /= S.sum(dim=1, keepdim=True)
    return S


def _count_block(S, b, dev, seed=0):
    """Raw Poisson counts of generator block b (rows [b*BLOCK, (b+1)*BLOCK))."""
    P = S.shape[0]
    g = torch.Generator(device=dev).manual_seed(seed * 1_000_003 + b + 1)
    gam = -torch.log(torch.rand((BLOCK, P), device=dev, generator=g).clamp_min_(1e-12))  # Exp(1)
    U = gam ** (1.0 / 0.3)                                       # skewed mixture weights
    U /= U.sum(dim=1, keepdim=True)
    lib = torch.empty(BLOCK, device=dev).log_normal_(float(np.log(2000.0)), 0.35, generator=g)
    # U @ S as P rank-1 updates (elementwise kernels), not a library GEMM: the kernel
    # summary of a profiled run then holds only the factorisation's own GEMMs
    lam = torch.zeros((BLOCK, S.shape[1]), device=dev)
    for k in range(P):
        lam.addcmul_(U[:, k:k + 1], S[k:k + 1])
    lam *= lib[:, None]
    return torch.poisson(lam, generator=g)


def device_counts(N, G, P, r0, r1, dev, comm, seed=0):
    """Rows [r0, r1) of the planted-program matrix, scaled to global unit variance."""
    S = _programs(G, P, dev, seed)
    X = torch.empty((r1 - r0, G), device=dev, dtype=torch.float32)
    b0 = r0 // BLOCK
    for b in range(b0, (r1 + BLOCK - 1) // BLOCK):
        lo, hi = max(r0, b * BLOCK), min(r1, (b + 1) * BLOCK)
        cnt = _count_block(S, b, dev, seed)
        X[lo - r0:hi - r0] = cnt[lo - b * BLOCK:hi - b * BLOCK]
        del cnt
    stats = torch.zeros(2 * G, dtype=torch.float64, device=dev)
    for i in range(0, X.shape[0], BLOCK):          # float64 sums without a float64 copy of X
        xb = X[i:i + BLOCK].double()
        stats[:G] += xb.sum(dim=0)
        stats[G:] += (xb * xb).sum(dim=0)
        del xb
    comm.allreduce_(stats)
    mean = stats[:G] / N
    var = (stats[G:] / N - mean ** 2) * (N / max(N - 1, 1))
    sd = torch.sqrt(var.clamp_min(0)).float()
    sd[sd == 0] = 1.0
    X /= sd
    return X


def planes_only_counts(N, G, P, r0, r1, dev, comm, seed=0):
    """The same matrix as device_counts, held ONLY as split-GEMM planes (nmf.PlanesOnlyX):
    a statistics pass for the per-gene scale, then every planes pass regenerates the
    blocks -- the 200 GB fp32 matrix of 10M x 5k is never resident."""
    from cnmf_torch_amd.models.nmf import PlanesOnlyX, RowBlocks

    S = _programs(G, P, dev, seed)
    b0, b1 = r0 // BLOCK, (r1 + BLOCK - 1) // BLOCK
    stats = torch.zeros(2 * G, dtype=torch.float64, device=dev)
    for b in range(b0, b1):
        lo, hi = max(r0, b * BLOCK), min(r1, (b + 1) * BLOCK)
        xb = _count_block(S, b, dev, seed)[lo - b * BLOCK:hi - b * BLOCK].double()
        stats[:G] += xb.sum(dim=0)
        stats[G:] += (xb * xb).sum(dim=0)
        del xb
    comm.allreduce_(stats)
    mean = stats[:G] / N
    var = (stats[G:] / N - mean ** 2) * (N / max(N - 1, 1))
    sd = torch.sqrt(var.clamp_min(0)).float()
    sd[sd == 0] = 1.0

    def blocks():
        for b in range(b0, b1):
            lo, hi = max(r0, b * BLOCK), min(r1, (b + 1) * BLOCK)
            yield lo - r0, _count_block(S, b, dev, seed)[lo - b * BLOCK:hi - b * BLOCK] / sd
    return PlanesOnlyX(RowBlocks(r1 - r0, G, blocks, dev))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=1_000_000)
    ap.add_argument("--genes", type=int, default=2000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=25, help="replicates per step (per rank unless --dp)")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--dp", action="store_true", help="cell-sharded data parallel")
    ap.add_argument("--max-pass", type=int, default=20)
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="with --dp on ONE process: run rank 0's shard of an N-rank DP job, "
                         "collectives replaced by device copies (parallel.comm.EmulatedComm): "
                         "the per-rank step time, value = projected N-GPU job rate")
    ap.add_argument("--coll-latency-us", type=float, default=33.4,
                    help="--emulate-world: per-call latency of the one-shot xGMI collectives "
                         "(default: tools/xgmi_latency.py, 2 ranks on one GPU, the slowest "
                         "kind at 4 KB -- profiles/r5_xgmi_latency.json)")
    ap.add_argument("--link-gbps", type=float, default=153.0,
                    help="--emulate-world: xGMI bandwidth per link and direction, GB/s")
    ap.add_argument("--planes-only", action="store_true",
                    help="hold X only as split-GEMM planes (10M x 5k on one GPU: fp32 X "
                         "and its planes do not fit together)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    emu = a.emulate_world if (a.dp and world == 1 and a.emulate_world and a.emulate_world > 1) \
        else None
    if emu:
        from cnmf_torch_amd.parallel.comm import EmulatedComm

        comm = EmulatedComm(emu)
    else:
        comm = DistComm() if (world > 1 and a.dp) else LocalComm()
    N, G = a.cells, a.genes
    if emu:
        r0, r1 = 0, N // emu
    elif a.dp:
        r0, r1 = N * rank // world, N * (rank + 1) // world
    else:
        r0, r1 = 0, N
    t0 = time.perf_counter()
    X = (planes_only_counts if a.planes_only else device_counts)(N, G, a.k, r0, r1, dev, comm)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    opts = NMFOptions(n_components=a.k, tol=1e-4, online_chunk_size=5000,
                      online_chunk_max_iter=1000, online_max_pass=a.max_pass)
    solver = NMFBatchSolver(X, opts, comm=comm, row_offset=r0)
    np.random.seed(14)
    seeds = np.random.randint(1, 2 ** 31 - 1, size=(a.warmup + a.steps) * a.reps * world)
    for i in range(a.warmup):
        solver.run([int(s) for s in seeds[i * a.reps:(i + 1) * a.reps]])
    if world > 1:
        dist.barrier()
    if emu:         # count the timed steps' collectives only
        comm.bytes, comm.log = 0, []
        comm.calls = {k: 0 for k in comm.calls}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    passes = []
    for i in range(a.warmup, a.warmup + a.steps):
        if a.dp:   # every rank works on the same replicates (its own rows)
            mine = seeds[i * a.reps:(i + 1) * a.reps]
        else:      # replicate-parallel: each rank its own slice of the ledger
            blk = seeds[i * a.reps * world:(i + 1) * a.reps * world]
            mine = blk[rank::world]
        res = solver.run([int(s) for s in mine])
        _ = res.W.cpu()
        passes.append(float(np.mean(res.n_iter)))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_reps = a.reps * a.steps * (1 if a.dp else world)
    proj = None
    if emu:
        # collective term of the projection: per call the one-shot kernels' latency plus the
        # bytes each rank pulls over ONE of its 7 links (all 7 in parallel): all-reduce the
        # whole payload from every peer, reduce-scatter / all-gather 1 / world of it
        lat = a.coll_latency_us
        per_link = {"all_reduce": 1.0, "reduce_scatter": 1.0 / emu, "all_gather": 1.0 / emu}
        t_coll = sum(lat * 1e-6 + nb * per_link[k] / (a.link_gbps * 1e9) for k, nb in comm.log)
        n_steps_online = sum(1 for k, _ in comm.log if k == "reduce_scatter") or None
        proj = {
            "collectives_per_step": {k: v / a.steps for k, v in comm.calls.items()},
            "collective_bytes_per_step_per_rank": int(comm.bytes / a.steps),
            "online_steps_per_step": (n_steps_online / a.steps) if n_steps_online else None,
            "latency_us_per_call": lat, "link_gbps": a.link_gbps,
            "collective_s_per_step": round(t_coll / a.steps, 4),
            "compute_s_per_step": round(el / a.steps, 4),
            "value_with_collectives": round(total_reps / (el + t_coll), 4),
            # the fused DP step issues each exchange unit's collectives in the background
            # under the other unit's compute (models/nmf_dp.py): the bound when all of it
            # hides (compute and collectives then overlap fully)
            "value_overlapped_bound": round(total_reps / max(el, t_coll), 4),
            "exchange_units": getattr(solver, "dp_units", None),
            "collective_model": "latency + per-link bytes / link bandwidth per call; "
                                "value_with_collectives: serial with compute (no overlap), "
                                "value_overlapped_bound: fully hidden"}
    if rank == 0:
        print(json.dumps({
            "metric": "NMF replicates/sec (large N)", "value": round(total_reps / el, 4),
            "unit": "replicates/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "s_per_step": round(el / a.steps, 3), "mean_passes": round(float(np.mean(passes)), 2),
            "data_gen_s": round(t_gen, 2), "dtype": "fp32",
            "config": {"cells": N, "genes": G, "k": a.k, "replicates_per_step": a.reps * (
                1 if a.dp else world),
                "parallelism": (f"dp x{emu} emulated on one GPU (rank 0's shard; collectives "
                                f"replaced by device copies, {comm.bytes / max(1, a.steps + a.warmup) / 1e6:.1f} "
                                "MB per step per rank not timed)") if emu else
                f"{'dp' if a.dp else 'replicate'}x{world}",
                "hbm_gb_X_per_gpu": round(N * G * 4 / 1e9 / (emu or (world if a.dp else 1)), 2),
                "x_storage": "split-GEMM planes only" if a.planes_only else "fp32 + planes",
                "hbm_gb_peak": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)},
            "projection": proj,
            "data": "synthetic planted-program Poisson counts generated on device"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

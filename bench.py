#!/usr/bin/env python
"""Headline benchmark: NMF replicates/sec at K=10, n_iter=100 (BASELINE.json).

Config ("PBMC-scale"): a synthetic 10,000-cell x 2,000-HVG
normalised-counts matrix (planted programs, Poisson counts, per-gene unit-variance
scaling exactly as cNMF's norm_counts, cnmf.py:670-681), K = 10, and the reference's
factorize settings (cnmf.py:757-771): online MU, Frobenius, tol 1e-4, chunk 5000,
online_chunk_max_iter = max_NMF_iter = 1000, random init from the ledger seeds.

One *step* = factorising one ledger batch of ``--n-iter`` (default 100) replicates to
convergence -- the whole cNMF ``factorize`` work for that batch (init, every pass, every
inner solve, convergence checks; spectra copied back to the host as factorize persists
them).  ``value`` is whole-job replicates/sec.  ``--mode`` picks the multi-GPU scaling:

* ``weak`` (default): every rank factorises its own 100 replicates (round-robin ledger
  shard, as ``worker_filter``): the job does 100*N replicates per step.
* ``strong``: one 100-replicate ledger batch per step, dealt round-robin over the ranks.
* ``dp``: one 100-replicate batch per step solved by ALL ranks together on a
  chunk-interleaved cell shard of X (parallel.runner.dp_row_segments) with the
  per-step ``[dB | dA]`` statistics all-reduced on RCCL -- the config for matrices too
  large for one GPU (BASELINE config 4); same factorisation path as one GPU.

``--kmin/--kmax`` replace the single K by the K x n_iter grid of BASELINE config 2
(K = kmin..kmax, ``--n-iter`` replicates each) solved as ONE ragged batch per step.

``--schedule batch`` (default): each step solves its ledger batch ALONE, to the last
replicate -- exactly the work ``cnmf factorize`` does for a ledger of ``--n-iter``
replicates of K (one solver batch, cnmf.py:876-892), so ``value`` does not depend on
``--steps``.  ``--schedule stream``: the timed steps' ledger batches are fed, in order,
through ONE continuous-batching solve (NMFBatchSolver.run_stream: a fixed number of live
replicate slots per K, each refilled with the next waiting replicate when its replicate
converged), so the tail of one batch overlaps the next batch's first passes -- the rate of
a multi-batch job (a K grid or several ledgers in one process).  With the default
schedule, a single-K run at K <= 16 ALSO times that stream over the same replicates and
reports it as ``config.stream_value`` (with ``config.stream_replicates``); ``value`` stays
the per-batch rate.

Run: ``python bench.py [--gpus N --steps K --warmup W --mode weak|strong|dp]``.  N > 1
runs one process per GPU over RCCL (xGMI): either under ``torch.distributed.run`` (the
driver's form; ``WORLD_SIZE`` must then equal ``--gpus``, else the run fails), or, when
started without a launcher, bench.py starts ``torch.distributed.run`` itself as a CHILD
process (before any GPU call; never an exec) and exits with its return code.  The JSON
line carries the world size and backend the process group actually reported
(``config.rccl_world``, ``config.backend``).  A weak-scaling run with N > 1 also times the
strong-scaling form of the same step -- ONE ``--n-iter`` ledger batch dealt round-robin
over the ranks -- and reports it as ``config.strong_value`` (replicates/s, whole job).

Reference: the multi-worker factorize is GNU parallel over ``--worker-index``
(/root/reference/Extras/run_parallel.py:48-51) with the round-robin ``worker_filter``
(/root/reference/src/cnmf/cnmf.py:53-54, 876-880).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

BASELINE_REPS_PER_SEC = 0.5  # PBMC3k, 120 replicates in ~240 s (CPU, sklearn cNMF)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--genes", type=int, default=2000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iter", type=int, default=100, help="replicates per GPU per step")
    ap.add_argument("--seed", type=int, default=14)
    ap.add_argument("--algo", default="mu")
    ap.add_argument("--nmf-mode", default="online", choices=["online", "batch"])
    ap.add_argument("--mode", default="weak", choices=["weak", "strong", "dp"],
                    help="multi-GPU scaling mode (see module docstring)")
    ap.add_argument("--kmin", type=int, default=None)
    ap.add_argument("--kmax", type=int, default=None)
    ap.add_argument("--allreduce", default="rccl", choices=["rccl", "xgmi"],
                    help="dp mode: RCCL ring all-reduce or the one-shot xGMI peer-memory "
                         "all-reduce (parallel/xgmi.py)")
    ap.add_argument("--beta-loss", default="frobenius")
    ap.add_argument("--max-nmf-iter", type=int, default=1000)
    ap.add_argument("--batch-size", type=int, default=5000)
    ap.add_argument("--cpu", action="store_true", help="run on CPU (plumbing check)")
    ap.add_argument("--float-input", action="store_true",
                    help="non-count data: X + 0.5 U(0,1) (e.g. batch-corrected counts), which "
                         "the integer-count plane detection declines")
    ap.add_argument("--density", type=float, default=None,
                    help="keep only the largest DENSITY fraction of X's entries (the rest 0): "
                         "sparse-input runs (KL switches to the CSR kernels at <= 0.15)")
    ap.add_argument("--streams", type=int, default=1,
                    help="replicate groups solved concurrently on separate HIP streams")
    ap.add_argument("--schedule", default="batch", choices=["stream", "batch"],
                    help="batch: one solve per step (the factorize job); stream: continuous "
                         "batching over the timed steps' replicates (see module docstring)")
    ap.add_argument("--batch-live", type=int, default=None,
                    help="batch schedule: solve each step's batch with this many live slots "
                         "(continuous batching inside the one ledger batch)")
    ap.add_argument("--no-stream-value", action="store_true",
                    help="batch schedule: skip the extra continuous-batching timing")
    ap.add_argument("--live", type=int, default=None,
                    help="stream schedule: live replicate slots per K (default: one "
                         "co-resident round of the usage solve, NMFBatchSolver.stream_live)")
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="dp mode on ONE process: run rank 0's cell shard of an N-rank job "
                         "with every collective replaced by a device copy of its bytes "
                         "(parallel.comm.EmulatedComm) -- the per-rank step time of the "
                         "N-GPU DP job, collectives excluded; value = projected job rate")
    ap.add_argument("--share-gpu", action="store_true",
                    help="(testing) every rank on GPU 0: gloo process group, device "
                         "collectives on the one-shot xGMI kernels, no cooperative solves -- "
                         "RCCL takes one rank per GPU")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return _self_launch(args.gpus)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} "
              "ranks", file=sys.stderr, flush=True)
        return 2

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # device_count() does not initialise the GPU on this image; is_available() does
    if args.share_gpu:
        os.environ["CNMF_SOLVE_COOP"] = "0"
        os.environ["CNMF_ALLREDUCE"] = "xgmi"
        args.allreduce = "xgmi"
    if not args.cpu and not args.share_gpu and world > 1 and 0 < torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but only {torch.cuda.device_count()} GPUs visible",
              file=sys.stderr, flush=True)
        return 2
    use_cuda = torch.cuda.is_available() and not args.cpu
    if use_cuda:
        if args.share_gpu:
            local_rank = 0
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:
        dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group(backend="nccl" if (use_cuda and not args.share_gpu) else "gloo",
                                device_id=dev if (use_cuda and not args.share_gpu) else None)

    from cnmf_torch_amd.models import nmf_graphs as _graphs
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.runner import dp_layout, dp_row_segments
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = normalized_counts_matrix(args.cells, args.genes, n_programs=args.k, seed=0)
    if args.float_input:
        X = (X + 0.5 * np.random.default_rng(1).random(X.shape)).astype(X.dtype)
    if args.density is not None:
        X[X < np.quantile(X, 1.0 - args.density)] = 0.0
    comm = row_map = schedule = None
    coll_calls = None
    emu = args.emulate_world if (args.mode == "dp" and world == 1 and args.emulate_world
                                 and args.emulate_world > 1) else None
    if args.mode == "dp" and (world > 1 or emu):
        segs = dp_row_segments(X.shape[0], args.batch_size, rank, emu or world)
        X = np.concatenate([X[a:b] for a, b in segs])
        row_map, schedule = dp_layout(segs)
        if emu:
            from cnmf_torch_amd.parallel.comm import EmulatedComm

            comm = EmulatedComm(emu)
        else:
            os.environ["CNMF_ALLREDUCE"] = args.allreduce
            comm = DistComm()
    Xd = torch.from_numpy(X).to(dev)
    opts = NMFOptions(n_components=args.k, init="random", beta_loss=args.beta_loss,
                      algo=args.algo, mode=args.nmf_mode, tol=1e-4,
                      online_chunk_size=args.batch_size,
                      online_chunk_max_iter=args.max_nmf_iter)
    solver = NMFBatchSolver(Xd, opts, comm=comm, row_map=row_map, schedule=schedule)

    # Ledger seeds exactly as cNMF.prepare draws them (cnmf.py:738-741), one ledger batch
    # per step; weak/strong: rank r takes every world-th replicate (worker_filter,
    # cnmf.py:53-54); dp: every rank takes all of them.
    grid = list(range(args.kmin, args.kmax + 1)) if args.kmin is not None else [args.k]
    per_batch = args.n_iter * len(grid)
    n_total = per_batch * world if args.mode == "weak" else per_batch
    nsteps = args.warmup + args.steps
    np.random.seed(args.seed)
    all_seeds = np.random.randint(low=1, high=(2 ** 31) - 1, size=n_total * nsteps)
    all_ks = np.tile(np.repeat(grid, args.n_iter), n_total // per_batch)

    def step(i: int, strong: bool = False):
        if strong:   # one ledger batch per step, dealt round-robin over the ranks
            seeds = all_seeds[i * per_batch:(i + 1) * per_batch]
            ks = all_ks[:per_batch]
        else:
            seeds = all_seeds[i * n_total:(i + 1) * n_total]
            ks = all_ks
        if args.mode != "dp":
            seeds, ks = seeds[rank::world], ks[rank::world]
        if args.batch_live is not None and args.mode != "dp":
            # the step's ledger batch through continuous batching INSIDE the batch (fewer
            # live slots than replicates; what factorize runs for that ledger)
            res = solver.run_stream([int(s) for s in seeds], ks=[int(k) for k in ks],
                                    live=args.batch_live, keep_usages=False)
        elif len(grid) == 1:
            res = solver.run_concurrent([int(s) for s in seeds], n_streams=args.streams)
        else:
            res = solver.run([int(s) for s in seeds], ks=[int(k) for k in ks])
        return res, to_host(res.W)   # factorize persists spectra (cnmf.py:889-892)

    # Spectra go to pinned host memory on a copy stream, as factorize overlaps its
    # replicate-file writes with the next batch's solve; the barrier that closes the timed
    # region synchronises the device, so every copy has landed inside it.
    copy_stream = torch.cuda.Stream(dev) if use_cuda else None
    host_bufs: dict = {}

    def to_host(W):
        if copy_stream is None:
            return W.cpu()
        key = tuple(W.shape)   # copies run in order on one stream: one buffer per shape
        buf = host_bufs.get(key)
        if buf is None:
            buf = torch.empty(W.shape, dtype=W.dtype, pin_memory=True)
            host_bufs[key] = buf
        copy_stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(copy_stream):
            buf.copy_(W, non_blocking=True)
        W.record_stream(copy_stream)    # W's memory is not reused before the copy ran
        return buf

    def barrier():
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    def max_over_ranks(sec: float) -> float:
        if world <= 1:
            return sec
        t = torch.tensor([sec], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # continuous batching where it pays: ranks K <= 16 (NMFBatchSolver.stream_live does
    # not stream wider ranks; a stream over every timed step's replicates would then be ONE
    # batch of all of them).  K = 20 / 30 measured 5,264-5,337 / 3,404-3,499 rep/s as that
    # single batch against 5,730 / 3,779-3,860 one batch per step (profiles/r5zp_*)
    stream_ok = args.mode != "dp" and args.streams == 1 and int(np.max(grid)) <= 16
    stream = args.schedule == "stream" and stream_ok
    held = []          # pinned spectra of finished replicates (factorize writes them out)

    def keep(ids, kk, host, ev):
        held.append((host, ev))

    def stream_steps(lo: int, hi: int, strong: bool = False):
        """Steps [lo, hi) as ONE continuous-batching solve (this rank's replicates)."""
        seeds, ks = [], []
        for i in range(lo, hi):
            if strong:
                s_, k_ = all_seeds[i * per_batch:(i + 1) * per_batch], all_ks[:per_batch]
            else:
                s_, k_ = all_seeds[i * n_total:(i + 1) * n_total], all_ks
            seeds += [int(v) for v in s_[rank::world]]
            ks += [int(v) for v in k_[rank::world]]
        held.clear()
        return solver.run_stream(seeds, ks=ks, live=args.live, keep_usages=False,
                                 on_result=keep)

    n_chunks = -(-args.cells // args.batch_size)
    passes, h_sweeps, w_sweeps = [], [], []

    def record(res):
        passes.append(float(np.mean(res.n_iter)))
        # inner MU sweeps per (replicate, pass, chunk) -- the solve kernels' work unit
        for key, acc in (("h_inner_iters", h_sweeps), ("w_inner_iters", w_sweeps)):
            it = np.asarray(res.stats.get(key, []), dtype=np.float64)
            if it.size:
                acc.append(float(np.mean(it / np.maximum(res.n_iter, 1) / n_chunks)))

    stream_info = None
    captures_timed = None
    if stream:
        if args.warmup:
            stream_steps(0, args.warmup)
        barrier()
        t0 = time.perf_counter()
        res = stream_steps(args.warmup, nsteps)
        if res.stats.get("stream_slots") is None:      # fell back to per-batch solves
            to_host(res.W)
        record(res)
        stream_info = {"slots": res.stats.get("stream_slots"),
                       "stagings": res.stats.get("stream_stagings"),
                       "passes": res.stats.get("stream_passes"),
                       "host_wait_s": res.stats.get("stream_host_wait_s"),
                       "host_stage_s": res.stats.get("stream_host_stage_s")}
    else:
        for i in range(args.warmup):
            if i == args.warmup - 1 and comm is not None and hasattr(comm, "record"):
                comm.record = []      # the collectives of one whole step (dp mode)
            step(i)
            if comm is not None and getattr(comm, "record", None) is not None:
                coll_calls, comm.record = comm.record, None
        barrier()
        t0 = time.perf_counter()
        cap0 = _graphs.CAPTURES[0]
        for i in range(args.warmup, nsteps):
            res, _ = step(i)
            record(res)
        captures_timed = _graphs.CAPTURES[0] - cap0
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps
    reps_per_sec = n_total * args.steps / elapsed

    # the multi-batch rate of the same replicates (continuous batching), beside the per-batch
    # value: timed separately, after the headline region
    # dp mode: the recorded collective sequence of one step, replayed alone and timed
    # between barriers -- the measured collective term, beside the emulated projection
    coll_s = None
    if coll_calls:
        coll_s = comm.replay(coll_calls, reps=5)
    stream_value = stream_reps = None
    if (not stream and stream_ok and len(grid) == 1 and args.schedule == "batch"
            and not args.no_stream_value and use_cuda):
        if args.warmup:
            stream_steps(0, args.warmup)
        barrier()
        t1 = time.perf_counter()
        sres = stream_steps(args.warmup, nsteps)
        if sres.stats.get("stream_slots") is None:
            to_host(sres.W)
        barrier()
        el_st = max_over_ranks(time.perf_counter() - t1)
        stream_reps = n_total * args.steps
        stream_value = stream_reps / el_st

    strong_value = strong_ms = None
    if world > 1 and args.mode == "weak":
        # the same ledger batch per step, now split over the ranks (strong scaling)
        if stream:
            stream_steps(0, min(2, args.warmup), strong=True) if args.warmup else None
            barrier()
            t0 = time.perf_counter()
            stream_steps(args.warmup, nsteps, strong=True)
        else:
            for i in range(min(2, args.warmup)):
                step(i, strong=True)
            barrier()
            t0 = time.perf_counter()
            for i in range(args.warmup, nsteps):
                step(i, strong=True)
        barrier()
        el_s = max_over_ranks(time.perf_counter() - t0)
        strong_ms = 1000.0 * el_s / args.steps
        strong_value = per_batch * args.steps / el_s
    rccl_world = dist.get_world_size() if world > 1 else 1
    backend = dist.get_backend() if world > 1 else None
    if rank == 0:
        metric = "NMF replicates/sec (K=10, n_iter=100)" if grid == [10] and args.n_iter == 100 \
            else f"NMF replicates/sec (K={grid[0]}..{grid[-1]}, n_iter={args.n_iter})" \
            if len(grid) > 1 else f"NMF replicates/sec (K={args.k}, n_iter={args.n_iter})"
        par = {"weak": f"replicate-parallel x{world}",
               "strong": f"replicate-parallel x{world} (fixed {n_total}-replicate ledger)",
               "dp": f"cell-sharded DP x{emu or world} ("
                     + ("emulated: rank 0's shard on one GPU, collectives replaced by device "
                        "copies" if emu else
                        f"{'one-shot xGMI' if args.allreduce == 'xgmi' else 'RCCL'} "
                        "reduce-scatter / all-gather per online step") + ")"}[args.mode]
        out = {
            "metric": metric,
            "value": round(reps_per_sec, 3),
            "unit": "replicates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "weak" else "strong",
            "vs_baseline": round(reps_per_sec / BASELINE_REPS_PER_SEC, 2),
            "dtype": "fp32",
            "data": "synthetic (planted-program Poisson counts, unit-variance genes; random-init W,H)",
            "config": {
                "model": f"cNMF factorize: {args.nmf_mode} {args.algo.upper()} {args.beta_loss}, "
                         f"K={args.k if len(grid) == 1 else f'{grid[0]}..{grid[-1]}'}",
                "global_batch": n_total,
                "seq_len": None,
                "cells": args.cells,
                "genes": args.genes,
                "n_iter_per_gpu": args.n_iter,
                "parallelism": par,
                "scaling_mode": args.mode,
                "streams_per_gpu": args.streams,
                "schedule": ("continuous batching over the timed steps (run_stream): "
                             f"live slots per K {stream_info['slots']}, "
                             f"{stream_info['stagings']} ring stagings, "
                             f"{stream_info['passes']} passes; host blocked on counters "
                             f"{stream_info['host_wait_s']} s, staging "
                             f"{stream_info['host_stage_s']} s")
                if stream_info and stream_info["slots"] else "one solve per step",
                "device": "cpu" if not use_cuda else torch.cuda.get_device_name(dev),
                "mean_passes": round(float(np.mean(passes)), 2) if passes else None,
                "graph_captures_timed": captures_timed,
                "mean_sweeps_h_w": [round(float(np.mean(h_sweeps)), 1) if h_sweeps else None,
                                    round(float(np.mean(w_sweeps)), 1) if w_sweeps else None],
                "input": ("float (X + 0.5 U(0,1))" if args.float_input else "counts / std")
                + (f", density {float((X != 0).mean()):.3f}" if args.density is not None else ""),
                "rccl_world": rccl_world,
                "backend": backend,
                "stream_value": None if stream_value is None else round(stream_value, 3),
                "stream_replicates": stream_reps,
                "strong_value": None if strong_value is None else round(strong_value, 3),
                "strong_ms_per_step": None if strong_ms is None else round(strong_ms, 3),
                "strong_global_batch": per_batch if strong_value is not None else None,
            },
        }
        if coll_calls:
            out["config"]["collective_s_per_step"] = round(coll_s, 6)
            out["config"]["collective_calls_per_step"] = len(coll_calls)
            out["config"]["collective_bytes_per_step_per_rank"] = int(sum(
                ni * torch.tensor([], dtype=dt).element_size() for _, ni, _, dt in coll_calls))
            out["config"]["collective_timing"] = ("one warmup step's collectives replayed "
                                                  "alone, each waited for, between barriers")
        if emu:
            out["config"]["emulated_world"] = emu
            out["config"]["collective_bytes_per_step_per_rank"] = int(comm.bytes / nsteps)
            out["config"]["projection"] = ("value = replicates/s of the emulated-world DP job "
                                           "from rank 0's per-step compute time; collective "
                                           "time not included (payload above)")
        print(json.dumps(out), flush=True)
    if comm is not None and hasattr(comm, "close"):
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def _free_port() -> int:
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def _self_launch(n: int) -> int:
    """``--gpus N`` without a launcher: run ``torch.distributed.run`` (N ranks, one per GPU,
    rendezvous on 127.0.0.1) as a child process with the same arguments and return its
    exit code.  Nothing here has touched the GPU (the parent never imports torch), and the
    parent waits instead of exec'ing."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())

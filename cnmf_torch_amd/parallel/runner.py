"""Multi-GPU stage drivers.

One process per GPU (``torchrun --nproc-per-node N``), ``torch.distributed`` with
backend ``nccl`` (RCCL over xGMI) for device work, ``gloo`` on CPU:

* ``distributed_factorize`` -- replicate parallelism: every rank takes a round-robin
  share of each K's replicates (ranks get the same K-mix, so batches stay balanced),
  solves them as device batches and writes its spectra files; a barrier closes the
  stage.  No collectives during the solves -- seeds are per replicate, so spectra are
  bit-identical to a single-GPU run of the same ledger.
* ``dp_factorize`` -- cell-sharded data parallelism for matrices too big for one GPU:
  rank r holds a contiguous row block of norm_counts, every replicate batch runs on all
  ranks with the per-step ``[dB | dA]`` statistics all-reduced (one RCCL call per
  online step), rank 0 writes the (replicated) spectra.
* ``distributed_consensus`` / ``distributed_k_selection`` -- K parallelism for the
  post-factorize stages: each rank takes a round-robin share of the Ks.
* fault tolerance: a restart with ``skip_completed_runs=True`` re-shards only the
  incomplete ledger rows over the surviving world size (resume by ledger, §5.3).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .comm import DistComm, LocalComm
from .ledger import shard_by_k


def init_distributed(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env vars; returns (comm, device)."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(dev)
    if world <= 1:
        return LocalComm(), dev
    if not dist.is_initialized():
        dist.init_process_group(backend=backend or ("nccl" if use_cuda else "gloo"),
                                device_id=dev if use_cuda else None)
    return DistComm(), dev


def _incomplete_jobs(obj, run_params, skip_completed_runs: bool, comm=None):
    """Ledger rows still to solve.  Under several ranks the list is rank 0's: a rank that
    looked later could see files a faster rank has already written in THIS run, deal
    itself a different shard, and leave replicates that no rank solves."""
    if not skip_completed_runs:
        return list(range(len(run_params)))
    done = [os.path.exists(obj.paths["iter_spectra"] % (int(k), int(i)))
            for k, i in zip(run_params["n_components"], run_params["iter"])]
    jobs = [i for i, d in enumerate(done) if not d]
    if comm is not None and comm.is_distributed:
        jobs = comm.all_gather_object(jobs)[0]
    return jobs


def distributed_factorize(obj, skip_completed_runs: bool = False, replicate_batch=None,
                          save_usages: bool = False, backend: str | None = None, verbose=True,
                          gather_spectra: bool = False):
    """Replicate-parallel factorize.  ``gather_spectra``: the replicate spectra also go to
    rank 0 by all-gather (RCCL) and rank 0 writes every K's merged spectra -- what
    ``combine`` would assemble from the files; the per-replicate
    files are still written as the durable checkpoint."""
    from ..utils.io import load_df_from_npz

    comm, dev = init_distributed(backend)
    run_params = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    jobs = _incomplete_jobs(obj, run_params, skip_completed_runs, comm)
    mine = shard_by_k(run_params, jobs, comm.rank, comm.world_size)
    collect = {} if gather_spectra else None
    obj.factorize_jobs(mine, worker_label=comm.rank, device=dev,
                       replicate_batch=replicate_batch, save_usages=save_usages,
                       verbose=verbose, run_params=run_params, collect=collect)
    if gather_spectra:
        gather_merged_spectra(obj, comm, collect, run_params, dev)
    comm.barrier()
    return comm


def gather_merged_spectra(obj, comm, collect: dict, run_params, dev) -> None:
    """Every K's replicate spectra onto rank 0 with one all-gather per K, then rank 0
    writes ``merged_spectra`` exactly as ``combine_nmf`` would (rows by iteration,
    ``iter%d_topic%d`` labels, gene columns).  Replicates solved in an earlier run (a
    resume) are not in memory: rank 0 reads their files, as combine does; a K with a
    replicate missing everywhere is left to ``combine``."""
    import pandas as pd

    from ..api import _load_npz_arrays
    from ..utils.io import NPZ_TMP_LEVEL, save_df_to_npz

    genes = collect.get("genes")
    genes_all = comm.all_gather_object(None if genes is None else list(genes))
    genes = next((g for g in genes_all if g is not None), None)
    if genes is None:
        return
    G = len(genes)
    tdev = dev if comm.is_distributed and getattr(comm, "backend", "") == "nccl" \
        else torch.device("cpu")
    ks = sorted(set(int(k) for k in run_params.n_components))
    for k in ks:
        its = sorted(int(i) for i in run_params.iter[run_params.n_components == k])
        mine = [it for it in its if (k, it) in collect]
        n_max = comm.allreduce_max_int(len(mine))
        buf = torch.zeros((max(n_max, 1), k, G), dtype=torch.float32, device=tdev)
        ids = torch.full((max(n_max, 1),), -1, dtype=torch.int64, device=tdev)
        for j, it in enumerate(mine):
            buf[j] = torch.from_numpy(np.ascontiguousarray(collect[(k, it)]))
            ids[j] = it
        parts = comm.all_gather_(buf)
        id_parts = comm.all_gather_(ids)
        if comm.rank != 0:
            continue
        got = {}
        for b, i in zip(parts, id_parts):
            for j, it in enumerate(i.cpu().tolist()):
                if it >= 0:
                    got[it] = b[j]
        rows = []
        for it in its:
            if it in got:
                rows.append(got[it].cpu().numpy())
                continue
            fn = obj.paths["iter_spectra"] % (k, it)
            if not os.path.exists(fn):
                rows = None
                break
            data, _, cols = _load_npz_arrays(fn)
            if not np.array_equal(np.asarray(cols).astype(str), np.asarray(genes).astype(str)):
                rows = None
                break
            rows.append(np.asarray(data, dtype=np.float32))
        if rows is None:
            continue
        index = ["iter%d_topic%d" % (it, t + 1) for it in its for t in range(k)]
        merged = pd.DataFrame(np.concatenate(rows, axis=0), index=index,
                              columns=np.asarray(genes))
        save_df_to_npz(merged, obj.paths["merged_spectra"] % k, level=NPZ_TMP_LEVEL)


def distributed_consensus(obj, ks, density_threshold=0.5, local_neighborhood_size=0.30,
                          show_clustering=True, build_ref=True, kmeans_backend="auto",
                          backend: str | None = None):
    """Consensus over the ranks.  With at least as many Ks as ranks: K parallelism (rank r
    runs ``consensus`` for ``ks[r::world]`` on its own GPU; every K writes its own
    artifacts, so the ranks share no files).  With fewer Ks than ranks (typically the one
    chosen K): every K runs on ALL ranks with its all-gene passes (TPM spectra refit, OLS
    gene scores over G_all) sharded by gene blocks -- tensor / gene-axis parallelism."""
    comm, dev = init_distributed(backend)
    ks = sorted(ks)
    if len(ks) >= comm.world_size or comm.world_size == 1:
        for k in ks[comm.rank::comm.world_size]:
            obj.consensus(k, density_threshold, local_neighborhood_size, show_clustering,
                          build_ref, close_clustergram_fig=True, kmeans_backend=kmeans_backend,
                          device=dev)
    else:
        for k in ks:
            obj.consensus(k, density_threshold, local_neighborhood_size,
                          show_clustering and comm.rank == 0, build_ref,
                          close_clustergram_fig=True, kmeans_backend=kmeans_backend, device=dev,
                          comm=comm)
    comm.barrier()
    return comm


def distributed_k_selection(obj, kmeans_backend="auto", backend: str | None = None):
    """K-parallel ``k_selection_plot``: stats per K on every rank, rank 0 writes."""
    comm, dev = init_distributed(backend)
    stats = obj.k_selection_plot(close_fig=True, kmeans_backend=kmeans_backend, comm=comm,
                                 device=dev)
    comm.barrier()
    return stats


def row_block(n_rows: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced row block of ``rank`` (first n % world ranks get one more)."""
    base, extra = divmod(n_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def dp_row_segments(n_rows: int, chunk: int, rank: int, world: int,
                    align: int = 8) -> list[tuple[int, int]]:
    """Global row segments held by ``rank`` in a chunk-interleaved cell shard: every
    online chunk [s*c, (s+1)*c) is split over ALL ranks (boundaries rounded down to
    ``align`` rows), so online step s on every rank works on its slice of the SAME global
    chunk and the all-reduced statistics of the step are exactly the single-GPU chunk's.
    The factorisation path is therefore independent of the world size, and every rank
    is busy in every step."""
    c = max(1, int(chunk))
    segs = []
    for a in range(0, n_rows, c):
        b = min(n_rows, a + c)
        n = b - a

        def cut(r):
            if r <= 0:
                return a
            if r >= world:
                return b
            return a + (n * r // world) // align * align

        segs.append((cut(rank), cut(rank + 1)))
    return segs


def dp_layout(segments):
    """(row_map [(local_a, local_b, global_a)], online schedule [[(local_a, local_b)]])
    of a rank's segments, one step per global chunk."""
    row_map, sched, off = [], [], 0
    for a, b in segments:
        n = max(0, b - a)
        row_map.append((off, off + n, a))
        sched.append([(off, off + n)])
        off += n
    return row_map, sched


def dp_factorize(obj, skip_completed_runs: bool = False, replicate_batch=None,
                 save_usages: bool = False, backend: str | None = None, verbose=True):
    """Cell-sharded factorize: every rank holds a chunk-interleaved shard of norm_counts
    (dp_row_segments) and all ranks solve every replicate batch together, all-reducing
    the [dB | dA] statistics once per online step; rank 0 writes the spectra."""
    from ..utils.h5ad import h5ad_shape
    from ..utils.io import load_df_from_npz, load_yaml

    comm, dev = init_distributed(backend)
    run_params = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    jobs = _incomplete_jobs(obj, run_params, skip_completed_runs, comm)
    n_rows, _ = h5ad_shape(obj.paths["normalized_counts"])
    chunk = int(load_yaml(obj.paths["nmf_run_parameters"]).get("online_chunk_size", 5000))
    segs = dp_row_segments(n_rows, chunk, comm.rank, comm.world_size)
    obj.factorize_jobs(jobs, worker_label=comm.rank, device=dev,
                       replicate_batch=replicate_batch, save_usages=save_usages,
                       verbose=verbose and comm.rank == 0, run_params=run_params,
                       comm=comm if comm.world_size > 1 else None, row_segments=segs)
    # a one-shot xGMI all-reduce that gave up on a peer leaves each rank with its own
    # partial statistics: fail the stage (every solver run also checks before returning)
    check = getattr(comm, "check", None)
    if check is not None:
        check()
    comm.barrier()
    close = getattr(comm, "close", None)
    if close is not None:       # collective: unmaps the xGMI peer workspaces, if any
        close()
    return comm

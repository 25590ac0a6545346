"""Replicate-ledger sharding (C4 ``worker_filter``, cnmf.py:53-54).

The ledger (one row per (K, iter, seed)) is the unit of work distribution.  Seeds are
per replicate, so any assignment of rows to workers/ranks yields identical spectra;
only throughput changes.  ``worker_filter`` keeps the reference's round-robin rule;
``shard_by_k`` keeps each rank's rows grouped by K so they batch well on one GPU.
"""
from __future__ import annotations

from collections import OrderedDict


def worker_filter(iterable, worker_index: int, total_workers: int):
    """Items whose position i satisfies (i - worker_index) % total_workers == 0."""
    return (p for i, p in enumerate(iterable) if (i - worker_index) % total_workers == 0)


def group_by_k(run_params, jobs) -> "OrderedDict[int, list[int]]":
    out: OrderedDict[int, list[int]] = OrderedDict()
    for idx in jobs:
        out.setdefault(int(run_params.iloc[idx]["n_components"]), []).append(int(idx))
    return out


def shard_by_k(run_params, jobs, rank: int, world: int) -> list[int]:
    """Round-robin inside every K group so each rank gets ~n_iter/world replicates of
    every K (balanced batches, the same K-mix on every GPU)."""
    mine: list[int] = []
    for _, idxs in group_by_k(run_params, jobs).items():
        mine.extend(list(worker_filter(idxs, rank, world)))
    return mine

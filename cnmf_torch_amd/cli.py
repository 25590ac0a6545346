"""``cnmf`` command line (C29, cnmf.py:1387-1470) -- same sub-commands and flags.

Restores ``--worker-index`` (documented in the reference's Stepwise_Guide.md:49-57 but
commented out at cnmf.py:1430) and gives ``--total-workers`` its documented meaning for
``factorize`` (number of workers sharing the ledger); for ``prepare`` it still maps to
``n_jobs`` as in the reference.  Under ``torchrun`` (WORLD_SIZE > 1) ``factorize``
shards the ledger over ranks automatically, one rank per GPU.

Additions: ``--algo``/``--mode`` (prepare), ``--replicate-batch``, ``--device``,
``--save-usages`` (factorize), ``--kmeans-backend``, ``--no-build-reference``
(consensus), ``--skip-missing-files`` (combine).
"""
from __future__ import annotations

import argparse
import os
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="cnmf")
    p.add_argument("command", type=str,
                   choices=["prepare", "factorize", "combine", "consensus", "k_selection_plot"])
    p.add_argument("--name", type=str, nargs="?", default="cNMF",
                   help="[all] Name for analysis. All output will be placed in [output-dir]/[name]/...")
    p.add_argument("--output-dir", type=str, nargs="?", default=".",
                   help="[all] Output directory. All output will be placed in [output-dir]/[name]/...")
    p.add_argument("-c", "--counts", type=str,
                   help="[prepare] Input (cell x gene) counts matrix as .h5ad, .mtx, df.npz, or tab delimited text file")
    p.add_argument("-k", "--components", type=int, nargs="+",
                   help='[prepare] Number of components (k) for matrix factorization. Several can be specified with "-k 8 9 10"')
    p.add_argument("-n", "--n-iter", type=int, default=100,
                   help="[prepare] Number of factorization replicates")
    p.add_argument("--total-workers", type=int, default=-1,
                   help="[all] Total number of workers to distribute jobs to")
    p.add_argument("--worker-index", type=int, default=None,
                   help="[factorize] Index of current worker (the first worker should have index 0)")
    p.add_argument("--use_gpu", action="store_true", default=False, help="[prepare] Whether to use GPU.")
    p.add_argument("--seed", type=int, default=None, help="[prepare] Seed for pseudorandom number generation")
    p.add_argument("--genes-file", type=str, default=None,
                   help="[prepare] File containing a list of genes to include, one gene per line.")
    p.add_argument("--numgenes", type=int, default=2000,
                   help="[prepare] Number of high variance genes to use for matrix factorization.")
    p.add_argument("--tpm", type=str, default=None,
                   help="[prepare] Pre-computed (cell x gene) TPM values as df.npz or tab separated txt file.")
    p.add_argument("--max-nmf-iter", type=int, default=1000,
                   help="[prepare] Max number of iterations per individual NMF run (default 1000)")
    p.add_argument("--beta-loss", type=str, default="frobenius",
                   choices=["frobenius", "kullback-leibler", "itakura-saito"],
                   help="[prepare] Loss function for NMF (default frobenius)")
    p.add_argument("--init", type=str, default="random", choices=["random", "nndsvd"],
                   help="[prepare] Initialization algorithm for NMF (default random)")
    p.add_argument("--densify", dest="densify", action="store_true", default=False,
                   help="[prepare] Treat the input data as non-sparse (default False)")
    p.add_argument("--batch_size", type=int, default=5000,
                   help="[prepare] Size of batch for online NMF learning.")
    p.add_argument("--algo", type=str, default="mu", choices=["mu", "hals", "halsvar", "bpp"],
                   help="[prepare] NMF update rule (addition; reference fixes mu)")
    p.add_argument("--mode", type=str, default="online", choices=["online", "batch"],
                   help="[prepare] NMF mode (addition; reference fixes online)")
    p.add_argument("--skip-completed-runs", action="store_true", default=False,
                   help="[factorize] Skip previously completed runs.")
    p.add_argument("--replicate-batch", type=int, default=None,
                   help="[factorize] Replicates solved together per launch (default: auto)")
    p.add_argument("--device", type=str, default=None, help="[factorize/consensus] torch device override")
    p.add_argument("--dp", action="store_true", default=False,
                   help="[factorize] cell-sharded data parallelism under torchrun: every rank "
                        "holds a shard of the cells, all ranks solve every replicate with the "
                        "statistics all-reduced on RCCL (for matrices too big for one GPU); "
                        "default under torchrun is replicate parallelism")
    p.add_argument("--save-usages", action="store_true", default=False,
                   help="[factorize] Also persist per-replicate usages (iter_usages files)")
    p.add_argument("--gather-spectra", action="store_true", default=False,
                   help="[factorize] under torchrun (replicate parallel): all-gather every "
                        "replicate's spectra onto rank 0 over RCCL and write the merged "
                        "spectra there (what combine assembles from the files)")
    p.add_argument("--skip-missing-files", action="store_true", default=False,
                   help="[combine] Ignore missing replicate files")
    p.add_argument("--local-density-threshold", type=float, default=0.5,
                   help="[consensus] Threshold for the local density filtering (0, 2]")
    p.add_argument("--local-neighborhood-size", type=float, default=0.30,
                   help="[consensus] Fraction of the number of replicates to use as nearest neighbors")
    p.add_argument("--show-clustering", dest="show_clustering", action="store_true",
                   help="[consensus] Produce a clustergram figure summarizing the spectra clustering")
    p.add_argument("--build-reference", dest="build_reference", action="store_true", default=True,
                   help="[consensus] Generates a reference spectra for use in starCAT")
    p.add_argument("--no-build-reference", dest="build_reference", action="store_false",
                   help="[consensus] Do not build the starCAT reference")
    p.add_argument("--kmeans-backend", type=str, default="auto",
                   choices=["auto", "sklearn", "device"],
                   help="[consensus] auto (device on GPU, else sklearn), sklearn (the "
                        "reference's exact KMeans) or device (batched GPU k-means)")
    return p


def _prepare_kwargs(args) -> dict:
    return dict(counts_fn=args.counts, components=args.components, n_iter=args.n_iter,
                densify=args.densify, tpm_fn=args.tpm, seed=args.seed,
                beta_loss=args.beta_loss, max_NMF_iter=args.max_nmf_iter,
                num_highvar_genes=args.numgenes, genes_file=args.genes_file, init=args.init,
                total_workers=args.total_workers, use_gpu=args.use_gpu,
                batch_size=args.batch_size, algo=args.algo, mode=args.mode)


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    from .api import cNMF

    obj = cNMF(output_dir=args.output_dir, name=args.name)
    if args.command == "prepare":
        # one stage per process: no later stage here could read a device mirror of the
        # files (utils.resident)
        os.environ.setdefault("CNMF_RESIDENT_BYTES", "0")
        comm = None
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:     # under torchrun: cell-sharded
            from .parallel.runner import init_distributed

            comm, _ = init_distributed()
        # (no background prewarm: the later stages run in other processes)
        obj.prepare(comm=comm, prewarm=False, **_prepare_kwargs(args))
    elif args.command == "factorize":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if args.dp:
            from .parallel.runner import dp_factorize

            dp_factorize(obj, skip_completed_runs=args.skip_completed_runs,
                         replicate_batch=args.replicate_batch, save_usages=args.save_usages)
        elif world > 1 and args.worker_index is None:
            from .parallel.runner import distributed_factorize

            distributed_factorize(obj, skip_completed_runs=args.skip_completed_runs,
                                  replicate_batch=args.replicate_batch,
                                  save_usages=args.save_usages,
                                  gather_spectra=args.gather_spectra)
        else:
            wi = args.worker_index if args.worker_index is not None else 0
            tw = args.total_workers if (args.worker_index is not None and args.total_workers > 0) else 1
            obj.factorize(worker_i=wi, total_workers=tw,
                          skip_completed_runs=args.skip_completed_runs, device=args.device,
                          replicate_batch=args.replicate_batch, save_usages=args.save_usages)
    elif args.command == "combine":
        obj.combine(components=args.components, skip_missing_files=args.skip_missing_files)
    elif args.command == "consensus":
        from .utils.io import load_df_from_npz

        if args.components is None:
            rp = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
            ks = sorted(set(int(k) for k in rp.n_components))
        else:
            ks = args.components
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            from .parallel.runner import distributed_consensus

            distributed_consensus(obj, ks, args.local_density_threshold,
                                  args.local_neighborhood_size, args.show_clustering,
                                  args.build_reference, kmeans_backend=args.kmeans_backend)
        else:
            for k in ks:
                obj.consensus(k, args.local_density_threshold, args.local_neighborhood_size,
                              args.show_clustering, args.build_reference,
                              close_clustergram_fig=True, kmeans_backend=args.kmeans_backend,
                              device=args.device, wait_figures=False)
    elif args.command == "k_selection_plot":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            from .parallel.runner import distributed_k_selection

            distributed_k_selection(obj, kmeans_backend=args.kmeans_backend)
        else:
            obj.k_selection_plot(close_fig=True, kmeans_backend=args.kmeans_backend,
                                 device=args.device, wait_figures=False)
    # every K's clustergram rendered while the next K computed: finish them before exit
    from .utils.plotting import flush_figures

    flush_figures()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Whole-pipeline driver (C39; reference Extras/run_parallel.py:16-66).

The reference shells out to ``cnmf.py prepare``, GNU ``parallel`` over
``--worker-index 0..n-1`` for ``factorize`` (a flag its own CLI had removed), then
``combine`` and ``k_selection_plot``.  Here the factorize stage is one process per GPU:

* ``--gpus N`` (N > 1): ``torch.distributed.run --nproc-per-node N -m cnmf_torch_amd
  factorize`` -- each rank takes a deterministic slice of the replicate ledger and
  batches its replicates through the HIP solver (RCCL only for the final barrier);
* ``--gpus 1``: a single in-process factorize;
* ``k_selection_plot`` and ``consensus`` run K-parallel over min(N, #K) ranks;
* ``--workers N`` (no torchrun): N plain worker processes with ``--worker-index``, each
  pinned to one device via HIP_VISIBLE_DEVICES -- the reference's shared-filesystem
  pattern, useful when ranks must not share a process group.

Usage::

    python -m cnmf_torch_amd.run_parallel --output-dir out --name run -c counts.h5ad \\
        -k 6 7 8 9 --n-iter 100 --gpus 8 --seed 5
"""
from __future__ import annotations

import argparse
import glob
import os
import socket
import subprocess
import time
import sys


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(cmd: list[str], env=None) -> None:
    print(" ".join(cmd), flush=True)
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        raise SystemExit(f"command failed with exit code {rc}: {' '.join(cmd)}")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="cnmf-run-parallel")
    p.add_argument("--name", type=str, default="cNMF")
    p.add_argument("--output-dir", type=str, default=".")
    p.add_argument("-c", "--counts", type=str, required=True)
    p.add_argument("-k", "--components", type=int, nargs="+", default=[10])
    p.add_argument("-n", "--n-iter", type=int, default=100)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--numgenes", type=int, default=None)
    p.add_argument("--genes-file", type=str, default=None)
    p.add_argument("--tpm", type=str, default=None)
    p.add_argument("--beta-loss", type=str, default=None)
    p.add_argument("--max-nmf-iter", type=int, default=None)
    p.add_argument("--batch_size", type=int, default=None)
    p.add_argument("--gpus", type=int, default=1, help="ranks for torchrun factorize")
    p.add_argument("--workers", type=int, default=None,
                   help="independent --worker-index processes instead of torchrun")
    p.add_argument("--dp", action="store_true",
                   help="cell-sharded data parallel factorize over --gpus ranks (one matrix "
                        "too big for one GPU) instead of replicate parallelism")
    p.add_argument("--keep-iterations", action="store_true",
                   help="keep cnmf_tmp/*.iter_*.df.npz after combine (reference deletes them)")
    p.add_argument("--local-density-threshold", type=float, default=None,
                   help="also run consensus at this threshold for every K")
    return p


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    py = sys.executable
    base = ["--output-dir", a.output_dir, "--name", a.name]
    prep = [py, "-m", "cnmf_torch_amd", "prepare"] + base + ["-c", a.counts, "-k"] + [
        str(k) for k in a.components] + ["-n", str(a.n_iter)]
    for flag, val in (("--seed", a.seed), ("--numgenes", a.numgenes),
                      ("--genes-file", a.genes_file), ("--tpm", a.tpm),
                      ("--beta-loss", a.beta_loss), ("--max-nmf-iter", a.max_nmf_iter),
                      ("--batch_size", a.batch_size)):
        if val is not None:
            prep += [flag, str(val)]
    _run(prep)

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t_factorize = time.time()
    if a.workers:
        procs = []
        for w in range(a.workers):
            e = dict(env)
            if a.gpus and a.gpus > 0:
                e["HIP_VISIBLE_DEVICES"] = str(w % a.gpus)
            cmd = [py, "-m", "cnmf_torch_amd", "factorize"] + base + [
                "--worker-index", str(w), "--total-workers", str(a.workers)]
            print(" ".join(cmd), flush=True)
            procs.append(subprocess.Popen(cmd, env=e))
        bad = [p.args for p in procs if p.wait() != 0]
        if bad:
            raise SystemExit(f"{len(bad)} factorize worker(s) failed")
    elif a.gpus > 1:
        # replicate parallel: the spectra also reach rank 0 by all-gather, which writes
        # the merged spectra (combine below then only fills in what is missing)
        _run([py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
              "-m", "cnmf_torch_amd", "factorize"] + base +
             (["--dp"] if a.dp else ["--gather-spectra"]), env=env)
    elif a.dp:
        _run([py, "-m", "cnmf_torch_amd", "factorize", "--dp"] + base, env=env)
    else:
        _run([py, "-m", "cnmf_torch_amd", "factorize"] + base, env=env)

    merged = [os.path.join(a.output_dir, a.name, "cnmf_tmp",
                           "%s.spectra.k_%d.merged.df.npz" % (a.name, k))
              for k in sorted(set(a.components))]
    if not all(os.path.exists(m) and os.path.getmtime(m) >= t_factorize for m in merged):
        _run([py, "-m", "cnmf_torch_amd", "combine"] + base)
    if not a.keep_iterations:
        pattern = os.path.join(a.output_dir, a.name, "cnmf_tmp", "*.iter_*.df.npz")
        for fn in glob.glob(pattern):
            os.remove(fn)
    # k-selection and consensus are K-parallel: one rank per GPU, Ks dealt round-robin
    n_k = len(set(a.components))
    kpar = min(a.gpus or 1, n_k) if not a.workers else 1
    launch = [py, "-m", "cnmf_torch_amd"]
    if kpar > 1:
        launch = [py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={kpar}",
                  "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                  "-m", "cnmf_torch_amd"]
    _run(launch + ["k_selection_plot"] + base, env=env)
    if a.local_density_threshold is not None:
        if kpar > 1:
            launch[launch.index("--master-port") + 1] = str(_free_port())
        _run(launch + ["consensus"] + base +
             ["--local-density-threshold", str(a.local_density_threshold)], env=env)
    return 0


if __name__ == "__main__":
    sys.exit(main())

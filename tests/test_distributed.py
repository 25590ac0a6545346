"""Multi-process tests on the gloo backend (world size 2, 3 and 8, CPU) -- the
fake-cluster strategy of SURVEY.md §4 item 4: cell-sharded DP == single process (same
schedule), replicate-parallel == serial, bit for bit where the math allows.  The world-8
cases use the driver's 8-GPU world with uneven shards: fewer replicates than ranks (ranks
that own none), R mod 8 != 0, and cell shards of unequal length."""
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

import dist_workers as W
from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix, simulate_counts


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args, timeout: float | None = None):
    """Run fn(rank, world, port, *args) on `world` processes; a run that has not finished
    within `timeout` seconds (CNMF_TEST_SPAWN_TIMEOUT, default 600) is terminated and
    fails the test -- a mismatched collective must not hang the suite silently."""
    import time

    if timeout is None:
        timeout = float(os.environ.get("CNMF_TEST_SPAWN_TIMEOUT", "600"))
    for attempt in range(3):
        ctx = mp.start_processes(fn, args=(world, _port()) + args, nprocs=world, join=False,
                                 start_method="spawn")
        deadline = time.monotonic() + timeout
        try:
            while not ctx.join(timeout=5):
                if time.monotonic() > deadline:
                    for p in ctx.processes:
                        if p.is_alive():
                            p.terminate()
                    for p in ctx.processes:
                        p.join(10)
                    raise TimeoutError(f"{fn.__name__}: {world} ranks still running after "
                                       f"{timeout} s")
            return
        except mp.ProcessRaisedException as e:
            # the free port picked by _port() was taken by a parallel test before the
            # rendezvous bound it: a fresh port, not a test failure
            if "EADDRINUSE" not in str(e) or attempt == 2:
                raise


@pytest.mark.parametrize("allreduce", ["rccl", "xgmi"])
def test_comm_primitives(tmp_path, monkeypatch, allreduce):
    # CNMF_ALLREDUCE=xgmi only reroutes float32 DEVICE buffers: host tensors stay on gloo
    monkeypatch.setenv("CNMF_ALLREDUCE", allreduce)
    _spawn(W.comm_worker, 3, str(tmp_path))
    for r in range(3):
        t, s, m, n, last, async_ok = np.load(tmp_path / f"comm{r}.npy")
        assert t == 6.0 and abs(s - 4.5) < 1e-12 and m == 20 and n == 3 and last == 2
        assert async_ok == 1.0      # reduce_scatter_async / all_gather_into_async


def test_dp_exchange_units():
    """The DP fused step's exchange units: a K grid's groups (each group's collectives
    overlap the other groups' compute); a one-K batch stays one unit unless split into
    halves (off by default: measured slower)."""
    from cnmf_torch_amd.models import nmf_dp
    from cnmf_torch_amd.models.nmf_batch import _Group

    g = _Group(K=7, p0=0, n=9, r0=0, q0=0)
    assert nmf_dp._dp_units([g], 2) == [g]
    u = nmf_dp._dp_units([g], 2, split=True)
    assert [(x.p0, x.n, x.r0, x.q0) for x in u] == [(0, 5, 0, 0), (5, 4, 35, 245)]
    assert nmf_dp._dp_units([_Group(7, 0, 3, 0, 0)], 2, split=True) == [_Group(7, 0, 3, 0, 0)]
    two = [_Group(5, 0, 3, 0, 0), _Group(8, 3, 4, 15, 75)]
    assert nmf_dp._dp_units(two, 2, split=True) == two


@pytest.mark.parametrize("algo,mode,beta_loss", [("mu", "online", "frobenius"),
                                                 ("hals", "online", "frobenius"),
                                                 ("mu", "batch", "frobenius"),
                                                 ("mu", "batch", "kullback-leibler"),
                                                 ("mu", "online", "kullback-leibler")])
@pytest.mark.parametrize("world", [2, 3, pytest.param(8, id="8")])
def test_dp_solver_matches_single_process(tmp_path, algo, mode, beta_loss, world):
    """Chunk-interleaved cell sharding: every online step all-reduces the statistics of
    the SAME global chunk the single-process solver uses, so the DP factorisation equals
    the plain single-process one (fp64: to summation order) for any world size.  The one
    rank-local decision is the usages' inner stopping rule (its block objective covers
    the rank's slice of the chunk), so it is pinned to a fixed count here
    (online_h_tol < 0); test_dp_default_tolerances_close_to_single_process covers it."""
    if world == 8 and (algo, mode, beta_loss) not in (("mu", "online", "frobenius"),
                                                      ("mu", "batch", "kullback-leibler")):
        pytest.skip("world 8: one online and one batch case")
    X = normalized_counts_matrix(603, 120, n_programs=4, seed=1).astype(np.float64)
    K, seeds = 4, [5, 6, 7]
    kw = dict(algo=algo, mode=mode, online_chunk_size=100, online_max_pass=6, batch_max_iter=30,
              beta_loss=beta_loss, fp_precision="double", online_h_tol=-1.0,
              online_chunk_max_iter=12)
    _spawn(W.dp_solver_worker, world, X, K, seeds, kw, str(tmp_path))
    ref = NMFBatchSolver(torch.from_numpy(X), NMFOptions(n_components=K, **kw)).run(seeds)
    Ws = [np.load(tmp_path / f"W{r}.npy") for r in range(world)]
    for Wr in Ws[1:]:
        np.testing.assert_array_equal(Ws[0], Wr)    # W replicated bit-identically
    np.testing.assert_allclose(Ws[0], ref.W.numpy(), rtol=1e-8, atol=1e-12)
    rows = np.concatenate([np.load(tmp_path / f"rows{r}.npy") for r in range(world)])
    HT = np.concatenate([np.load(tmp_path / f"HT{r}.npy") for r in range(world)], axis=1)
    np.testing.assert_allclose(HT, ref.HT.numpy()[:, rows], rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(np.load(tmp_path / "err0.npy"), ref.err, rtol=1e-10)


def test_dp_default_tolerances_close_to_single_process(tmp_path):
    X = normalized_counts_matrix(1200, 150, n_programs=5, seed=2).astype(np.float64)
    K, seeds = 5, [1, 2, 3, 4]
    kw = dict(online_chunk_size=300, online_max_pass=20, fp_precision="double")
    _spawn(W.dp_solver_worker, 3, X, K, seeds, kw, str(tmp_path))
    ref = NMFBatchSolver(torch.from_numpy(X), NMFOptions(n_components=K, **kw)).run(seeds)
    np.testing.assert_allclose(np.load(tmp_path / "err0.npy"), ref.err, rtol=1e-2)


def test_dp_row_segments_cover_every_row_once():
    from cnmf_torch_amd.parallel.runner import dp_row_segments

    for n, c, w in [(10000, 5000, 8), (603, 100, 3), (7, 5000, 4), (12345, 777, 5),
                    (10001, 5000, 3)]:
        rows = np.concatenate([np.arange(a, b) for r in range(w)
                               for a, b in dp_row_segments(n, c, r, w)])
        assert np.array_equal(np.sort(rows), np.arange(n))
        if c % 8:
            continue
        for r in range(w):   # every local block starts 8-aligned (split-GEMM k offsets)
            off = 0
            for a, b in dp_row_segments(n, c, r, w):
                assert off % 8 == 0 or b <= a
                off += b - a


@pytest.fixture(scope="module")
def prepared(tmp_path_factory):
    d = tmp_path_factory.mktemp("dist")
    Xc, cells, genes = simulate_counts(400, 200, 4, seed=9, sparse=False)
    fn = d / "counts.df.npz"
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), str(fn))
    return d, str(fn)


@pytest.mark.parametrize("mode,world", [("replicate", 2), ("dp", 2), ("replicate", 8),
                                        ("dp", 8)])
def test_distributed_factorize_matches_serial(prepared, mode, world):
    """Replicate-parallel (worker_filter dealing, cnmf.py:53-54) and cell-sharded DP
    factorize == serial.  World 8: 6 replicates, so ranks 6 and 7 own none (replicate
    mode), and 400 cells in 150-cell chunks give every rank a shard of 18-19 cells of each
    chunk (DP)."""
    d, fn = prepared
    name = f"d_{mode}_{world}"
    obj = cNMF(output_dir=str(d), name=name)
    obj.prepare(fn, components=[3, 4], n_iter=3, seed=11, num_highvar_genes=120, batch_size=150)
    _spawn(W.factorize_worker, world, str(d), name, mode)
    par = {(k, i): load_df_from_npz(obj.paths["iter_spectra"] % (k, i)).values
           for k in (3, 4) for i in range(3)}
    serial = cNMF(output_dir=str(d), name=name + "_serial")
    serial.prepare(fn, components=[3, 4], n_iter=3, seed=11, num_highvar_genes=120, batch_size=150)
    serial.factorize()
    # DP at 8 ranks: each rank stops its usages' inner solve on the block objective of its
    # OWN ~19 cells of the chunk (the one rank-local decision of the DP schedule,
    # test_dp_solver_matches_single_process pins it and is exact at world 8), so the
    # iterates drift from the serial ones by more than summation order
    loose = mode == "dp" and world > 3
    for (k, i), v in par.items():
        ref = load_df_from_npz(serial.paths["iter_spectra"] % (k, i)).values
        # replicate-parallel: same solves; DP: the chunk-interleaved shard all-reduces the
        # same global chunks as the serial solver -- both differ by fp32 summation only
        if loose:
            cos = (v * ref).sum(1) / np.linalg.norm(v, axis=1) / np.linalg.norm(ref, axis=1)
            assert cos.min() > 0.99, (k, i, cos)
        else:
            np.testing.assert_allclose(v, ref, rtol=2e-3, atol=1e-6)
    if mode == "dp":
        from cnmf_torch_amd.utils.timing import read_jsonl

        e_dp = {(r["k"], r["iter"]): r["err"] for r in read_jsonl(obj.paths["replicate_log"])}
        e_se = {(r["k"], r["iter"]): r["err"] for r in read_jsonl(serial.paths["replicate_log"])}
        assert set(e_dp) == set(e_se)
        for key in e_dp:
            np.testing.assert_allclose(e_dp[key], e_se[key], rtol=1e-2 if loose else 1e-4,
                                       err_msg=str(key))


def test_gathered_merged_spectra_equal_file_combine(prepared):
    """distributed_factorize(gather_spectra=True): the replicate spectra reach rank 0 by
    all-gather and rank 0 writes every K's merged spectra -- identical (values, row labels,
    gene columns) to what combine assembles from the per-replicate files.  A replicate
    solved in an earlier run (resume) is taken from its file."""
    import os

    d, fn = prepared
    name = "gathered"
    obj = cNMF(output_dir=str(d), name=name)
    obj.prepare(fn, components=[3, 4], n_iter=3, seed=13, num_highvar_genes=120, batch_size=150)
    # one replicate solved "earlier": only its file exists when the ranks start
    rp = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    obj.factorize_jobs([0], run_params=rp, verbose=False)
    _spawn(W.factorize_worker, 2, str(d), name, "gather")
    gathered = {k: load_df_from_npz(obj.paths["merged_spectra"] % k) for k in (3, 4)}
    for k in (3, 4):
        os.remove(obj.paths["merged_spectra"] % k)
    obj.combine()
    for k in (3, 4):
        ref = load_df_from_npz(obj.paths["merged_spectra"] % k)
        assert list(gathered[k].index) == list(ref.index)
        assert list(gathered[k].columns) == list(ref.columns)
        np.testing.assert_array_equal(gathered[k].values, ref.values)


def test_k_parallel_consensus_and_k_selection_match_serial(prepared):
    """distributed_consensus / distributed_k_selection (Ks dealt over 2 gloo ranks) write
    the same artifacts as the serial stages."""
    import glob

    d, fn = prepared
    obj = cNMF(output_dir=str(d), name="kpar")
    obj.prepare(fn, components=[3, 4, 5], n_iter=4, seed=5, num_highvar_genes=120,
                batch_size=150)
    obj.factorize()
    obj.combine()
    keys = ("consensus_spectra", "consensus_usages", "gene_spectra_score",
            "gene_spectra_tpm", "starcat_spectra")
    ser_stats = obj.k_selection_plot(close_fig=True)
    ser = {}
    for k in (3, 4, 5):
        obj.consensus(k, 0.5, show_clustering=False, close_clustergram_fig=True)
        ser.update({(key, k): load_df_from_npz(obj.paths[key] % (k, "0_5")).values
                    for key in keys})
    # drop every serial output (and the density caches) so the ranks recompute them
    outs = [obj.paths["k_selection_stats"]] + [obj.paths[key] % (k, "0_5")
                                               for key in keys for k in (3, 4, 5)]
    outs += glob.glob(str(d / "kpar" / "cnmf_tmp" / "*local_density_cache*"))
    for f in outs:
        os.remove(f)
    _spawn(W.consensus_worker, 2, str(d), "kpar", [3, 4, 5])
    par_stats = load_df_from_npz(obj.paths["k_selection_stats"])
    np.testing.assert_allclose(par_stats.values.astype(float),
                               ser_stats.values.astype(float), rtol=1e-6)
    for (key, k), v in ser.items():
        np.testing.assert_allclose(load_df_from_npz(obj.paths[key] % (k, "0_5")).values, v,
                                   rtol=1e-6, atol=1e-12, err_msg=f"{key} k={k}")


def test_rank_failure_then_resume_on_a_different_world_size(prepared):
    """a rank dies mid-factorize; a restart with --skip-completed-runs
    semantics on a different world size re-shards only the missing replicates, and the
    final spectra equal a serial run (seeds are per replicate, not per rank)."""
    d, fn = prepared
    name = "fault"
    obj = cNMF(output_dir=str(d), name=name)
    obj.prepare(fn, components=[3, 4], n_iter=3, seed=5, num_highvar_genes=100)
    _spawn(W.fault_worker, 2, str(d), name, 1)
    st1 = (d / "status1.txt").read_text()
    assert "injected failure" in st1
    done = [os.path.exists(obj.paths["iter_spectra"] % (k, i)) for k in (3, 4) for i in range(3)]
    assert 0 < sum(done) < 6
    obj.update_nmf_iter_params()
    _spawn(W.resume_worker, 3, str(d), name)
    serial = cNMF(output_dir=str(d), name=name + "_serial")
    serial.prepare(fn, components=[3, 4], n_iter=3, seed=5, num_highvar_genes=100)
    serial.factorize(verbose=False)
    for k in (3, 4):
        for i in range(3):
            a = load_df_from_npz(obj.paths["iter_spectra"] % (k, i)).values
            b = load_df_from_npz(serial.paths["iter_spectra"] % (k, i)).values
            np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-6)


def _write_10x(d, X, cells, genes):
    import scipy.io
    import scipy.sparse as sp

    os.makedirs(d, exist_ok=True)
    scipy.io.mmwrite(os.path.join(d, "matrix.mtx"), sp.coo_matrix(np.asarray(X).T))
    with open(os.path.join(d, "features.tsv"), "w") as fh:
        fh.write("".join(f"{g}\t{g}\tGene Expression\n" for g in genes))
    with open(os.path.join(d, "barcodes.tsv"), "w") as fh:
        fh.write("".join(f"{c}\n" for c in cells))
    return os.path.join(d, "matrix.mtx")


@pytest.mark.parametrize("fmt,world", [("h5ad_sparse", 3), ("npz_dense", 3), ("txt_sparse", 3),
                                       ("mtx_sparse", 3), ("npz_densify", 3),
                                       ("h5ad_sparse", 8), ("npz_dense", 8)])
def test_sharded_prepare_matches_single_process(tmp_path, fmt, world):
    """Cell-sharded prepare over 3 gloo ranks -- each rank reads ONLY its cells (partial
    h5ad reads, streamed 10x mtx / npz member / TSV lines), gene statistics from exact
    integer moments all-reduced, row blocks handed to rank 0's writer in messages of at
    most CNMF_PREPARE_CHUNK_BYTES -- writes artifacts bit-identical to the single-process
    prepare."""
    from cnmf_torch_amd.utils.anndata_lite import AnnData
    from cnmf_torch_amd.utils.h5ad import read_h5ad, write_h5ad

    sparse = fmt in ("h5ad_sparse", "mtx_sparse")
    Xc, cells, genes = simulate_counts(500, 300, 4, seed=21, sparse=sparse)
    if fmt == "h5ad_sparse":
        fn = str(tmp_path / "counts.h5ad")
        write_h5ad(fn, AnnData(X=Xc, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
    elif fmt == "mtx_sparse":
        fn = _write_10x(str(tmp_path / "tenx"), Xc.toarray(), cells, genes)
    elif fmt == "txt_sparse":
        fn = str(tmp_path / "counts.txt")
        pd.DataFrame(np.asarray(Xc), index=cells, columns=genes).to_csv(fn, sep="\t")
    else:
        fn = str(tmp_path / "counts.df.npz")
        save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    bound = 4096
    kw = dict(components=[3, 4], n_iter=3, seed=7, num_highvar_genes=120,
              densify=fmt == "npz_densify")
    _spawn(W.prepare_worker, world, str(tmp_path), "sh", fn, dict(kw, _chunk_bytes=bound))
    for r in range(1, world):
        m = int(np.load(tmp_path / f"maxmsg{r}.npy")[0])
        assert 0 < m <= bound, m
    ser = cNMF(output_dir=str(tmp_path), name="se")
    ser.prepare(fn, **kw)
    sh = cNMF(output_dir=str(tmp_path), name="sh")
    assert open(sh.paths["nmf_genes_list"]).read() == open(ser.paths["nmf_genes_list"]).read()
    sa, sb = load_df_from_npz(sh.paths["tpm_stats"]), load_df_from_npz(ser.paths["tpm_stats"])
    assert sa.values.dtype == sb.values.dtype
    np.testing.assert_array_equal(sa.values, sb.values)
    for key in ("normalized_counts", "tpm"):
        a, b = read_h5ad(sh.paths[key]), read_h5ad(ser.paths[key])
        xa = a.X.toarray() if hasattr(a.X, "toarray") else a.X
        xb = b.X.toarray() if hasattr(b.X, "toarray") else b.X
        assert xa.dtype == xb.dtype
        np.testing.assert_array_equal(xa, xb)
        assert list(a.obs.index) == list(b.obs.index) and list(a.var.index) == list(b.var.index)
    pa = load_df_from_npz(sh.paths["nmf_replicate_parameters"])
    pb = load_df_from_npz(ser.paths["nmf_replicate_parameters"])
    assert pa.equals(pb)


@pytest.mark.parametrize("world", [3, 8])
def test_gene_sharded_consensus_matches_serial(prepared, world):
    """One K on 3 / 8 gloo ranks: the TPM spectra refit and the OLS gene scores over G_all
    are sharded by whole refit chunks (tensor / gene-axis parallelism) and all-gathered;
    the artifacts equal the serial consensus (at 8 ranks some ranks own no gene block)."""
    d, fn = prepared
    obj = cNMF(output_dir=str(d), name=f"tp{world}")
    obj.prepare(fn, components=[4], n_iter=4, seed=8, num_highvar_genes=120, batch_size=60)
    obj.factorize(verbose=False)
    obj.combine()
    keys = ("consensus_spectra", "consensus_usages", "gene_spectra_score", "gene_spectra_tpm",
            "starcat_spectra")
    obj.consensus(4, 0.5, show_clustering=False, close_clustergram_fig=True)
    ser = {key: load_df_from_npz(obj.paths[key] % (4, "0_5")) for key in keys}
    for key in keys:
        os.remove(obj.paths[key] % (4, "0_5"))
    _spawn(W.tp_consensus_worker, world, str(d), f"tp{world}", 4)
    for key in keys:
        got = load_df_from_npz(obj.paths[key] % (4, "0_5"))
        assert list(got.columns) == list(ser[key].columns), key
        np.testing.assert_allclose(got.values, ser[key].values, rtol=1e-5, atol=1e-9,
                                   err_msg=key)


def test_incomplete_jobs_are_rank0s_list(prepared):
    """Resume under several ranks: every rank deals its shard from rank 0's list of
    unfinished replicates, not from its own later look at the files (a faster rank's
    fresh files would otherwise shift the dealing and leave replicates unsolved)."""
    from cnmf_torch_amd.parallel.runner import _incomplete_jobs

    d, fn = prepared
    obj = cNMF(output_dir=str(d), name="jobs_view")
    obj.prepare(fn, components=[3], n_iter=4, seed=2, num_highvar_genes=100, batch_size=150)
    rp = load_df_from_npz(obj.paths["nmf_replicate_parameters"])

    class _Comm:
        is_distributed = True

        def all_gather_object(self, obj_):
            return [[0, 1, 2, 3], obj_]          # rank 0 looked before any file existed

    obj.factorize_jobs([0], run_params=rp, verbose=False)
    assert _incomplete_jobs(obj, rp, True) == [1, 2, 3]
    assert _incomplete_jobs(obj, rp, True, _Comm()) == [0, 1, 2, 3]


def test_solver_raises_when_the_communicator_reports_a_failed_collective():
    """A communicator whose collective gave up (the xGMI all-reduce's timeout flag) makes
    the solver raise before returning spectra a caller could persist."""
    import torch

    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.parallel.comm import LocalComm
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    class FailedComm(LocalComm):
        def check(self):
            raise RuntimeError("peer did not arrive")

    X = torch.from_numpy(normalized_counts_matrix(200, 40, n_programs=3, seed=1))
    solver = NMFBatchSolver(X, NMFOptions(n_components=3, online_chunk_size=100,
                                          online_max_pass=2), comm=FailedComm())
    with pytest.raises(RuntimeError, match="peer did not arrive"):
        solver.run([1, 2])


def test_nccl_comm_stages_host_tensors_through_the_device():
    """DistComm.allreduce_ of a HOST tensor under an RCCL ("nccl") group -- the sharded
    prepare's int64 moment digits -- is staged through the backend's device buffer:
    RCCL has no CPU backend.  The process group is faked; the staging copy must be what
    the collective sees, and the reduced values must land in the caller's tensor."""
    from cnmf_torch_amd.parallel.comm import DistComm

    seen = []

    class _FakeDist:
        def all_reduce(self, x, group=None, op=None):
            seen.append(x)
            x.mul_(2)

    c = DistComm.__new__(DistComm)
    c._dist, c.group, c.rank, c.world_size, c.backend, c._xgmi = _FakeDist(), None, 0, 2, \
        "nccl", None
    c._dev = lambda: torch.device("cpu")        # stands in for the rank's GPU
    t = torch.arange(5, dtype=torch.int64)
    c.allreduce_(t)
    assert len(seen) == 1 and seen[0] is not t
    assert t.tolist() == [0, 2, 4, 6, 8]

"""Multi-process tests on the gloo backend (world size 2-3, CPU) -- the fake-cluster
strategy of SURVEY.md §4 item 4: cell-sharded DP == single process (same schedule),
replicate-parallel == serial, bit for bit where the math allows."""
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
from cnmf_torch_amd.parallel.runner import row_block
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix, simulate_counts


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    mp.spawn(fn, args=(world, _port()) + args, nprocs=world, join=True)


def test_comm_primitives(tmp_path):
    _spawn(W.comm_worker, 3, str(tmp_path))
    for r in range(3):
        t, s, m, n, last = np.load(tmp_path / f"comm{r}.npy")
        assert t == 6.0 and abs(s - 4.5) < 1e-12 and m == 20 and n == 3 and last == 2


@pytest.mark.parametrize("algo,mode,beta_loss", [("mu", "online", "frobenius"),
                                                 ("hals", "online", "frobenius"),
                                                 ("mu", "batch", "frobenius"),
                                                 ("mu", "batch", "kullback-leibler"),
                                                 ("mu", "online", "kullback-leibler")])
def test_dp_solver_matches_single_process(tmp_path, algo, mode, beta_loss):
    X = normalized_counts_matrix(603, 120, n_programs=4, seed=1)
    K, seeds, world = 4, [5, 6, 7], 2
    kw = dict(algo=algo, mode=mode, online_chunk_size=100, online_max_pass=6, batch_max_iter=30,
              beta_loss=beta_loss)
    _spawn(W.dp_solver_worker, world, X, K, seeds, kw, str(tmp_path))
    # single-process emulation of the sharded schedule: step s = {rank0 chunk s, rank1 chunk s}
    blocks = [row_block(X.shape[0], r, world) for r in range(world)]
    c = kw["online_chunk_size"]
    n_steps = max((b - a + c - 1) // c for a, b in blocks)
    sched = [[(a + s * c, min(b, a + (s + 1) * c)) for a, b in blocks] for s in range(n_steps)]
    ref = NMFBatchSolver(torch.from_numpy(X), NMFOptions(n_components=K, **kw),
                         schedule=sched).run(seeds)
    W0 = np.load(tmp_path / "W0.npy")
    W1 = np.load(tmp_path / "W1.npy")
    np.testing.assert_array_equal(W0, W1)          # W replicated bit-identically on all ranks
    np.testing.assert_allclose(W0, ref.W.numpy(), rtol=2e-3, atol=1e-5)
    HT = np.concatenate([np.load(tmp_path / "HT0.npy"), np.load(tmp_path / "HT1.npy")], axis=1)
    np.testing.assert_allclose(HT, ref.HT.numpy(), rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(np.load(tmp_path / "err0.npy"), ref.err, rtol=1e-4)


@pytest.fixture(scope="module")
def prepared(tmp_path_factory):
    d = tmp_path_factory.mktemp("dist")
    Xc, cells, genes = simulate_counts(400, 200, 4, seed=9, sparse=False)
    fn = d / "counts.df.npz"
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), str(fn))
    return d, str(fn)


@pytest.mark.parametrize("mode", ["replicate", "dp"])
def test_distributed_factorize_matches_serial(prepared, mode):
    d, fn = prepared
    name = f"d_{mode}"
    obj = cNMF(output_dir=str(d), name=name)
    obj.prepare(fn, components=[3, 4], n_iter=3, seed=11, num_highvar_genes=120, batch_size=150)
    _spawn(W.factorize_worker, 2, str(d), name, mode)
    par = {(k, i): load_df_from_npz(obj.paths["iter_spectra"] % (k, i)).values
           for k in (3, 4) for i in range(3)}
    serial = cNMF(output_dir=str(d), name=name + "_serial")
    serial.prepare(fn, components=[3, 4], n_iter=3, seed=11, num_highvar_genes=120, batch_size=150)
    serial.factorize()
    for (k, i), v in par.items():
        ref = load_df_from_npz(serial.paths["iter_spectra"] % (k, i)).values
        if mode == "replicate":
            np.testing.assert_allclose(v, ref, rtol=2e-3, atol=1e-6)  # fp32 GEMM blocking only
    if mode == "dp":
        # DP changes the online step composition (one chunk per rank per step), so the
        # replicates take a different path; exact equivalence with the emulated schedule is
        # test_dp_solver_matches_single_process.  Here: same-quality factorisations.
        from cnmf_torch_amd.utils.timing import read_jsonl

        e_dp = {(r["k"], r["iter"]): r["err"] for r in read_jsonl(obj.paths["replicate_log"])}
        e_se = {(r["k"], r["iter"]): r["err"] for r in read_jsonl(serial.paths["replicate_log"])}
        assert set(e_dp) == set(e_se)
        for key in e_dp:
            assert 0.9 < e_dp[key] / e_se[key] < 1.1, (key, e_dp[key], e_se[key])


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

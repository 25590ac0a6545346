"""End-to-end CPU pipeline (BASELINE.json config 1: 1k cells x 500 genes, K=5, n_iter=5)
plus resume / worker sharding / CLI behaviour the reference never tested."""
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest
import torch

from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
from cnmf_torch_amd.utils.synthetic import simulate_counts


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def counts_file(tmp_path_factory):
    d = tmp_path_factory.mktemp("data")
    X, cells, genes, U, S = simulate_counts(1000, 500, 5, seed=3, sparse=False, return_truth=True)
    fn = d / "counts.df.npz"
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), str(fn))
    return str(fn), S, genes


@pytest.fixture(scope="module")
def run_dir(tmp_path_factory, counts_file):
    out = tmp_path_factory.mktemp("run")
    obj = cNMF(output_dir=str(out), name="sim")
    obj.prepare(counts_file[0], components=[4, 5, 6], n_iter=6, seed=14, num_highvar_genes=300,
                batch_size=400)
    obj.factorize(worker_i=0, total_workers=1)
    obj.combine()
    return obj


def test_factorize_outputs(run_dir):
    obj = run_dir
    for k in (4, 5, 6):
        for it in range(6):
            assert os.path.exists(obj.paths["iter_spectra"] % (k, it))
        merged = load_df_from_npz(obj.paths["merged_spectra"] % k)
        assert merged.shape[0] == 6 * k
        assert merged.index[0] == "iter0_topic1"
        assert (merged.values >= 0).all()
    log = [l for l in open(obj.paths["replicate_log"])]
    assert len(log) == 18


def test_consensus_artifacts_and_recovery(run_dir, counts_file):
    obj = run_dir
    obj.consensus(5, density_threshold=0.5, show_clustering=True, close_clustergram_fig=True)
    dt = "0_5"
    p = obj.paths
    for key in ("consensus_spectra", "consensus_usages", "gene_spectra_tpm", "gene_spectra_score",
                "starcat_spectra"):
        assert os.path.exists(p[key] % (5, dt)), key
    for key in ("consensus_spectra__txt", "consensus_usages__txt", "gene_spectra_tpm__txt",
                "gene_spectra_score__txt", "starcat_spectra__txt", "clustering_plot"):
        assert os.path.exists(p[key] % (5, dt)), key
    usage, scores, tpm_spectra, top = obj.load_results(5, 0.5, n_top_genes=20)
    assert usage.shape == (1000, 5)
    np.testing.assert_allclose(usage.sum(axis=1).values, 1.0, rtol=1e-6)
    assert top.shape == (20, 5)
    # planted programs are recovered: each true program matches a consensus GEP
    _, S_true, genes = counts_file
    gt = pd.DataFrame(S_true, columns=genes)
    est = tpm_spectra.T
    A = gt.values / np.linalg.norm(gt.values, axis=1, keepdims=True)
    B = est[gt.columns].values
    B = B / np.linalg.norm(B, axis=1, keepdims=True)
    sims = A @ B.T
    from scipy.optimize import linear_sum_assignment

    r, c = linear_sum_assignment(-sims)
    assert sims[r, c].min() > 0.9, sims[r, c]
    starcat = load_df_from_npz(p["starcat_spectra"] % (5, dt))
    assert list(starcat.index) == [f"GEP{i}" for i in range(1, 6)]
    # consensus builds the reference from the in-memory TPM spectra; the standalone call
    # re-reads the TSV as the reference does (cnmf.py:1273): identical bits
    obj.build_reference(5, 0.5)
    again = load_df_from_npz(p["starcat_spectra"] % (5, dt))
    assert again.equals(starcat)
    assert list(again.columns) == list(starcat.columns)


def test_k_selection(run_dir):
    stats = run_dir.k_selection_plot(close_fig=True)
    assert list(stats.k) == [4, 5, 6]
    assert os.path.exists(run_dir.paths["k_selection_plot"])
    assert (stats.prediction_error > 0).all()
    assert stats.silhouette.between(-1, 1).all()


def test_resume_and_worker_sharding(tmp_path, counts_file):
    obj = cNMF(output_dir=str(tmp_path), name="res")
    obj.prepare(counts_file[0], components=[5], n_iter=4, seed=1, num_highvar_genes=200)
    # worker 1 of 2 takes the odd ledger rows only
    obj.factorize(worker_i=1, total_workers=2)
    made = [os.path.exists(obj.paths["iter_spectra"] % (5, i)) for i in range(4)]
    assert made == [False, True, False, True]
    obj.update_nmf_iter_params()
    rp = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    assert rp["completed"].astype(bool).tolist() == made
    obj.factorize(skip_completed_runs=True)
    assert all(os.path.exists(obj.paths["iter_spectra"] % (5, i)) for i in range(4))


def test_replicate_batching_invariance(tmp_path, counts_file):
    """Same seed -> same spectra whether solved alone or inside a batch."""
    obj = cNMF(output_dir=str(tmp_path), name="inv")
    obj.prepare(counts_file[0], components=[5], n_iter=3, seed=2, num_highvar_genes=200)
    obj.factorize(replicate_batch=3)
    a = [load_df_from_npz(obj.paths["iter_spectra"] % (5, i)).values for i in range(3)]
    for i in range(3):
        os.remove(obj.paths["iter_spectra"] % (5, i))
    obj.factorize(replicate_batch=1)
    b = [load_df_from_npz(obj.paths["iter_spectra"] % (5, i)).values for i in range(3)]
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-6)


def test_fault_injection_then_resume(tmp_path, counts_file, monkeypatch):
    obj = cNMF(output_dir=str(tmp_path), name="fault")
    obj.prepare(counts_file[0], components=[5], n_iter=4, seed=3, num_highvar_genes=200)
    monkeypatch.setenv("CNMF_FAULT_AFTER_REPLICATES", "2")
    with pytest.raises(RuntimeError, match="injected failure"):
        obj.factorize(replicate_batch=4)
    monkeypatch.delenv("CNMF_FAULT_AFTER_REPLICATES")
    obj.update_nmf_iter_params()
    rp = load_df_from_npz(obj.paths["nmf_replicate_parameters"])
    assert int(rp["completed"].astype(bool).sum()) == 2
    obj.factorize(skip_completed_runs=True)
    obj.combine()
    assert load_df_from_npz(obj.paths["merged_spectra"] % 5).shape[0] == 20
    # no temp files left behind by atomic writes
    assert not [f for f in os.listdir(os.path.dirname(obj.paths["iter_spectra"]))
                if f.startswith(".tmp_")]


def test_combine_skip_missing(tmp_path, counts_file):
    obj = cNMF(output_dir=str(tmp_path), name="miss")
    obj.prepare(counts_file[0], components=[5], n_iter=3, seed=4, num_highvar_genes=200)
    obj.factorize(worker_i=0, total_workers=3)
    with pytest.raises(FileNotFoundError):
        obj.combine()
    obj.combine(skip_missing_files=True)
    assert load_df_from_npz(obj.paths["merged_spectra"] % 5).shape[0] == 5


def test_cli_end_to_end(tmp_path, counts_file):
    env = dict(os.environ, PYTHONPATH=ROOT)
    base = [sys.executable, "-m", "cnmf_torch_amd"]
    common = ["--output-dir", str(tmp_path), "--name", "cli"]

    def run(*a):
        r = subprocess.run(base + list(a) + common, env=env, capture_output=True, text=True,
                           timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout

    run("prepare", "-c", counts_file[0], "-k", "4", "5", "-n", "6", "--seed", "7",
        "--numgenes", "200")
    out = run("factorize", "--worker-index", "0", "--total-workers", "1")
    assert "[Worker 0]. Starting task 0." in out
    run("combine")
    run("consensus", "-k", "5", "--local-density-threshold", "2.0", "--show-clustering")
    run("k_selection_plot")
    d = tmp_path / "cli"
    assert (d / "cli.spectra.k_5.dt_2_0.consensus.txt").exists()
    assert (d / "cli.clustering.k_5.dt_2_0.png").exists()
    assert (d / "cli.k_selection.png").exists()


def test_device_kmeans_backend_on_cpu_matches_sklearn_partition():
    from sklearn.metrics import adjusted_rand_score

    from cnmf_torch_amd.models.consensus import kmeans, local_density, pairwise_distances

    rs = np.random.default_rng(1)
    centers = rs.normal(size=(4, 30)) * 4
    truth = rs.integers(0, 4, 300)
    X = centers[truth] + rs.normal(size=(300, 30))
    a = kmeans(torch.from_numpy(X), 4, backend="device")
    b = kmeans(X, 4, backend="sklearn")
    assert adjusted_rand_score(a, b) > 0.99
    D = pairwise_distances(torch.from_numpy(X))
    dens = local_density(D, 5).numpy()
    exp = np.sort(D.numpy(), axis=1)[:, :6].sum(1) / 5
    np.testing.assert_allclose(dens, exp)


def test_run_parallel_driver_with_workers(tmp_path):
    """C39: prepare -> N worker-index processes -> combine -> k_selection_plot."""
    Xc, cells, genes = simulate_counts(150, 80, 3, seed=3, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    cmd = [sys.executable, "-m", "cnmf_torch_amd.run_parallel", "--output-dir", str(tmp_path),
           "--name", "rp", "-c", fn, "-k", "3", "4", "-n", "4", "--seed", "2", "--numgenes", "50",
           "--workers", "2", "--gpus", "0"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    obj = cNMF(output_dir=str(tmp_path), name="rp")
    for k in (3, 4):
        merged = load_df_from_npz(obj.paths["merged_spectra"] % k)
        assert merged.shape == (4 * k, 50)
    assert not any("iter_" in f for f in os.listdir(os.path.join(str(tmp_path), "rp", "cnmf_tmp")))
    assert os.path.exists(obj.paths["k_selection_stats"])


def test_run_parallel_driver_with_torchrun_ranks(tmp_path):
    """C39 over torchrun (gloo on the CPU here, RCCL on GPUs): replicate-parallel
    factorize, then K-parallel k_selection_plot and consensus over 2 ranks."""
    Xc, cells, genes = simulate_counts(150, 80, 3, seed=3, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    cmd = [sys.executable, "-m", "cnmf_torch_amd.run_parallel", "--output-dir", str(tmp_path),
           "--name", "rt", "-c", fn, "-k", "3", "4", "5", "-n", "4", "--seed", "2",
           "--numgenes", "50", "--gpus", "2", "--local-density-threshold", "2.0"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    obj = cNMF(output_dir=str(tmp_path), name="rt")
    stats = load_df_from_npz(obj.paths["k_selection_stats"])
    assert list(stats["k"].astype(int)) == [3, 4, 5]
    for k in (3, 4, 5):
        assert load_df_from_npz(obj.paths["consensus_spectra"] % (k, "2_0")).shape == (k, 50)
        assert load_df_from_npz(obj.paths["consensus_usages"] % (k, "2_0")).shape == (150, k)


def test_replicate_manifest_detects_corruption(tmp_path):
    Xc, cells, genes = simulate_counts(120, 70, 3, seed=4, sparse=False)
    fn = str(tmp_path / "c.df.npz")
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    obj = cNMF(output_dir=str(tmp_path), name="man")
    obj.prepare(fn, components=[3], n_iter=3, seed=1, num_highvar_genes=40)
    obj.factorize(verbose=False)
    assert obj.verify_replicates() == []
    victim = obj.paths["iter_spectra"] % (3, 1)
    with open(victim, "r+b") as fh:
        fh.seek(40)
        fh.write(b"\x00\x01\x02")
    os.remove(obj.paths["iter_spectra"] % (3, 2))
    probs = {(p["iter"], p["problem"]) for p in obj.verify_replicates()}
    assert probs == {(1, "checksum mismatch"), (2, "missing")}


def test_cli_dp_factorize_over_torchrun_matches_serial(tmp_path):
    """`cnmf factorize --dp` under torchrun (2 gloo ranks here, RCCL on GPUs): the
    chunk-interleaved cell shard all-reduces the same chunks as a single process, so the
    replicate spectra equal a serial factorize to fp32 summation order."""
    Xc, cells, genes = simulate_counts(400, 120, 3, seed=6, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    objs = {}
    for name in ("dp", "serial"):
        obj = cNMF(output_dir=str(tmp_path), name=name)
        obj.prepare(fn, components=[3, 4], n_iter=2, seed=3, num_highvar_genes=60, batch_size=96)
        objs[name] = obj
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "cnmf_torch_amd", "factorize", "--output-dir", str(tmp_path), "--name", "dp",
           "--dp"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    objs["serial"].factorize(verbose=False)
    for k in (3, 4):
        for i in range(2):
            a = load_df_from_npz(objs["dp"].paths["iter_spectra"] % (k, i)).values
            b = load_df_from_npz(objs["serial"].paths["iter_spectra"] % (k, i)).values
            np.testing.assert_allclose(a, b, rtol=5e-3, atol=1e-6)


def test_figures_drawn_by_plot_worker_process(tmp_path):
    """Closed figures (CLI / pipeline) are drawn by a child process that imports matplotlib
    while the stage computes, and serves the later stages too: the stage process itself
    never imports pyplot."""
    Xc, cells, genes = simulate_counts(150, 80, 3, seed=3, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(Xc, index=cells, columns=genes), fn)
    code = f"""
import os, sys
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from cnmf_torch_amd import cNMF
o = cNMF(output_dir={repr(str(tmp_path))}, name="pw")
o.prepare({repr(fn)}, components=[3, 4], n_iter=10, seed=1, num_highvar_genes=50)
o.factorize(verbose=False); o.combine()
o.k_selection_plot(close_fig=True)
from cnmf_torch_amd.utils.plotting import _PlotProc
pid = _PlotProc._inst.proc.pid
o.consensus(3, 2.0, show_clustering=True, close_clustergram_fig=True)
assert _PlotProc._inst.proc.pid == pid      # one child, matplotlib imported once
assert 'matplotlib.pyplot' not in sys.modules
assert os.path.getsize(o.paths['k_selection_plot']) > 1000
assert os.path.getsize(o.paths['clustering_plot'] % (3, '2_0')) > 1000
print('ok')
"""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("MPLBACKEND", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_native_png_matches_matplotlib_pixels(tmp_path):
    """utils.plotting._save (Agg canvas at 250 dpi + the banded-deflate PNG writer, native
    and Python fallback) decodes to exactly the pixels of matplotlib's own savefig."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from PIL import Image

    from cnmf_torch_amd.utils import plotting

    rng = np.random.default_rng(0)
    n = 120
    D = rng.random((n, n))
    D = (D + D.T) / 2
    lab = pd.Series(rng.integers(1, 5, n), index=[f"s{i}" for i in range(n)])
    fig = plotting.clustergram(D, lab, pd.DataFrame(rng.random(n), columns=["local_density"]),
                               np.ones(n, bool), 0.5, str(tmp_path / "cg.png"))
    fig.savefig(str(tmp_path / "ref.png"), dpi=250)
    ref = np.asarray(Image.open(str(tmp_path / "ref.png")))
    got = np.asarray(Image.open(str(tmp_path / "cg.png")))
    assert got.shape == ref.shape and (got == ref).all()
    info = Image.open(str(tmp_path / "cg.png")).info
    assert abs(info["dpi"][0] - 250) < 0.1 and info["Software"].startswith("Matplotlib")
    # the pure-Python writer (used when the native module is missing)
    saved = sys.modules.get("cnmf_torch_amd.utils._npzio")
    sys.modules["cnmf_torch_amd.utils._npzio"] = None          # ImportError on import
    try:
        plotting.write_png_rgba(str(tmp_path / "py.png"), ref, 250, threads=3)
    finally:
        if saved is None:
            sys.modules.pop("cnmf_torch_amd.utils._npzio", None)
        else:
            sys.modules["cnmf_torch_amd.utils._npzio"] = saved
    assert (np.asarray(Image.open(str(tmp_path / "py.png"))) == ref).all()
    plt.close(fig)


def test_plot_worker_falls_back_when_the_child_dies(tmp_path):
    """A dead figure child is replaced for the next stage, and a job it never acknowledged
    is drawn in this process: figures are never lost."""
    from cnmf_torch_amd.utils.plotting import PlotWorker, _PlotProc

    w = PlotWorker()
    w.proc.proc.kill()
    w.proc.proc.wait()
    path = str(tmp_path / "ksel.png")
    w.submit("k_selection", path, k=np.array([3, 4]), silhouette=np.array([0.9, 0.8]),
             prediction_error=np.array([10.0, 9.0]))
    w.wait(timeout=60)
    assert os.path.getsize(path) > 1000
    w2 = PlotWorker()                         # a fresh child for the next stage
    assert w2.proc is _PlotProc._inst and w2.proc.proc.poll() is None
    path2 = str(tmp_path / "ksel2.png")
    w2.submit("k_selection", path2, k=np.array([3, 4]), silhouette=np.array([0.9, 0.8]),
              prediction_error=np.array([10.0, 9.0]))
    w2.wait(timeout=120)
    assert os.path.getsize(path2) > 1000


def test_gpu_rank_limit_is_routed_with_a_message(monkeypatch, tmp_path):
    """-k beyond what the native GPU kernels cover is announced at prepare (warning +
    log naming the limit) and routed to the eager PyTorch ops -- not a failed job.
    Frobenius MU and the beta-divergences cover every K (the rank-general paths beyond
    the tiled kernels), HALS 512."""
    import torch

    from cnmf_torch_amd import api

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    assert api.check_gpu_ranks([10, 130, 1000], "frobenius", "mu", use_gpu=True) == []
    assert api.check_gpu_ranks([10, 80, 300], "frobenius", "hals", use_gpu=True) == []
    with pytest.warns(RuntimeWarning, match=r"K=\[600\]: the native gfx950 kernels factorise K <= 512"):
        assert api.check_gpu_ranks([10, 600], "frobenius", "hals", use_gpu=True) == [600]
    assert api.check_gpu_ranks([40, 80], "kullback-leibler", "mu", use_gpu=True) == []
    assert api.check_gpu_ranks([60, 300], "itakura-saito", "mu", use_gpu=True) == []
    assert api.check_gpu_ranks([800], "frobenius", "bpp", use_gpu=True) == []  # torch linalg
    api.check_gpu_ranks([80], "kullback-leibler", "mu", use_gpu=False)     # CPU: any K
    api.check_gpu_ranks([64], "frobenius", "mu", use_gpu=True)


def test_prediction_error_caches_x_sq_per_tensor():
    """The ||X||^2 cache of a resident dense X is keyed by tensor identity: a second
    lookup with the same tensor must not compare tensors (api._XSQ)."""
    import torch

    from cnmf_torch_amd.api import _XSQ
    rng = np.random.default_rng(0)
    X = torch.as_tensor(rng.random((50, 20)), dtype=torch.float32)
    U, S = rng.random((50, 3)), rng.random((3, 20))
    want = float(((X.double().numpy() - U @ S) ** 2).sum())
    for _ in range(2):
        got = cNMF._prediction_error(X, U, S, torch.device("cpu"))
        assert abs(got - want) <= 1e-9 * want
    assert X in _XSQ


@pytest.mark.parametrize("n,c,seed", [(300, 5, 0), (257, 13, 1), (90, 2, 2)])
def test_silhouette_matches_sklearn_precomputed(n, c, seed):
    """consensus.silhouette (segmented per-row cluster sums, ops.seg_rowsum) ==
    sklearn.metrics.silhouette_score(metric='precomputed') on the same float64 distance
    matrix to 1e-10 -- singleton clusters included (score 0, as sklearn)."""
    from sklearn.metrics import silhouette_score

    from cnmf_torch_amd.models.consensus import pairwise_distances, silhouette

    rs = np.random.default_rng(seed)
    X = rs.random((n, 7)) + rs.integers(0, c, n)[:, None] * 0.5
    lab = rs.integers(0, c, n)
    lab[0] = c + 3                       # a singleton cluster with a non-contiguous label
    D = pairwise_distances(torch.from_numpy(X))
    got = silhouette(D, lab)
    want = silhouette_score(D.numpy(), lab, metric="precomputed")
    assert abs(got - want) <= 1e-10 * max(1.0, abs(want))


def test_prepare_with_h5ad_tpm_copies_it_in_the_background(tmp_path, counts_file):
    """An .h5ad tpm_fn is copied on a worker thread while prepare runs on the object read
    from the source: the copy is complete (byte-identical) when prepare returns, and the
    statistics / norm counts equal those of prepare computing the TPM itself."""
    from cnmf_torch_amd.models.hvg import compute_tpm
    from cnmf_torch_amd.utils.h5ad import write_h5ad
    from cnmf_torch_amd.utils.io import read_any

    tpm_fn = str(tmp_path / "tpm.h5ad")
    write_h5ad(tpm_fn, compute_tpm(read_any(counts_file[0], False)))
    out = {}
    for name, tfn in (("own", None), ("given", tpm_fn)):
        obj = cNMF(output_dir=str(tmp_path), name=name)
        obj.prepare(counts_file[0], components=[5], n_iter=2, seed=1, num_highvar_genes=200,
                    tpm_fn=tfn, prewarm=False)
        out[name] = obj
    with open(tpm_fn, "rb") as a, open(out["given"].paths["tpm"], "rb") as b:
        assert a.read() == b.read()
    for key in ("tpm_stats", "normalized_counts"):
        if key == "tpm_stats":
            x, y = (load_df_from_npz(o.paths[key]) for o in out.values())
            pd.testing.assert_frame_equal(x, y)
        else:
            x, y = (read_any(o.paths[key], False).X for o in out.values())
            np.testing.assert_array_equal(x.toarray(), y.toarray())

"""One-shot xGMI all-reduce (parallel/xgmi.py, csrc/kernels/xgmi_allreduce.hip).

The GPU box has one MI355X, so the ranks here are processes sharing that GPU: each maps
the others' workspaces through hipIpcOpenMemHandle exactly as across the GPUs of a node,
and the per-slice flag handshake is the same.  Compared against gloo's all-reduce of the
same buffers (2 ranks: a + b, the same float32 sum in either order)."""
import numpy as np
import pytest
import torch

import dist_workers as W
from test_distributed import _spawn
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

pytestmark = pytest.mark.gpu


def test_xgmi_allreduce_matches_gloo(tmp_path):
    _spawn(W.xgmi_worker, 2, str(tmp_path), timeout=150)
    r0, r1 = (np.load(tmp_path / f"xgmi{r}.npz") for r in range(2))
    n_calls = sum(1 for k in r0.files if k.startswith("err"))
    assert n_calls == 61
    for i in range(n_calls):
        assert r0[f"err{i}"] == 0.0 and r1[f"err{i}"] == 0.0, i
        np.testing.assert_array_equal(r0[f"sum{i}"], r1[f"sum{i}"])   # identical on ranks
    for r in (r0, r1):
        assert bool(r["comm_is_xgmi"])
        np.testing.assert_array_equal(r["comm"], np.full(10, 3.0, dtype=np.float32))
    assert bool(r0["timed_out"]) and bool(r1["timed_out"])     # every rank fails together
    # the workspace peers hand data over in is coherent across devices while kernels run:
    # uncached or fine-grained (hipPointerGetAttributes), never coarse-grained hipMalloc
    for r in (r0, r1):
        assert str(r["memory_kind"]) in ("uncached", "fine-grained"), r["memory_kind"]


def test_xgmi_dp_solve_matches_gloo_staged(tmp_path):
    """Cell-sharded DP online MU with the [dB | dA] all-reduce over peer memory == the same
    solve with the all-reduce staged through gloo (same float32 sums)."""
    X = normalized_counts_matrix(1200, 300, n_programs=5, seed=3)
    K, seeds = 5, [11, 12, 13, 14]
    kw = dict(online_chunk_size=200, online_max_pass=8, online_h_tol=-1.0,
              online_chunk_max_iter=10)
    for ar in ("xgmi", "rccl"):
        _spawn(W.xgmi_dp_worker, 2, X, K, seeds, kw, str(tmp_path), ar, timeout=150)
    assert bool(np.load(tmp_path / "used_xgmi0.npy"))
    assert not bool(np.load(tmp_path / "used_rccl0.npy"))
    Wx, Wg = np.load(tmp_path / "W_xgmi0.npy"), np.load(tmp_path / "W_rccl0.npy")
    np.testing.assert_array_equal(Wx, np.load(tmp_path / "W_xgmi1.npy"))
    np.testing.assert_allclose(Wx, Wg, rtol=1e-4, atol=1e-6)
    ref = NMFBatchSolver(torch.from_numpy(X).cuda(), NMFOptions(n_components=K, **kw)).run(seeds)
    np.testing.assert_allclose(np.load(tmp_path / "err_xgmi0.npy"), ref.err, rtol=1e-3)


def test_xgmi_reduce_scatter_all_gather_match_gloo(tmp_path):
    """One-shot reduce-scatter and all-gather (float32 and int16 bit patterns), mixed with
    all-reduces on one device call counter, == gloo's results bitwise on both ranks --
    eagerly and from a replayed HIP graph; DistComm routes both under
    CNMF_ALLREDUCE=xgmi."""
    _spawn(W.xgmi_rsag_worker, 2, str(tmp_path), timeout=150)
    for r in range(2):
        z = np.load(tmp_path / f"rsag{r}.npz")
        n = int(z["n"])
        assert n == 12
        for i in range(n):
            assert z[f"rs{i}"] == 0.0 and z[f"ag{i}"] == 0.0 and z[f"ar{i}"] == 0.0, i
            assert int(z[f"agi{i}"]) == 0, i
        for i in range(3):
            assert z[f"grs{i}"] == 0.0 and z[f"gag{i}"] == 0.0, i
        assert bool(z["comm_is_xgmi"])
        np.testing.assert_array_equal(z["comm_rs"], np.full(3, 3.0, dtype=np.float32))
        np.testing.assert_array_equal(z["comm_ag"], np.repeat([7, 8], 4).astype(np.int16))
        np.testing.assert_array_equal(z["comm_rs_async"], np.full(5, 6.0, dtype=np.float32))
        np.testing.assert_array_equal(z["comm_ag_async"],
                                      np.repeat([3, 4], 6).astype(np.int16))


@pytest.mark.parametrize("K,R", [(6, 7), (20, 6), ((5, 5, 5, 8, 8, 8, 8), 7)])
def test_dp_fused_reduce_scatter_step_matches_unfused(tmp_path, K, R):
    """Cell-sharded DP with the fused step -- reduce-scatter of dB and the per-slice
    partial Grams, each rank W-solving only its replicate chunk (R not a multiple of the
    world: a padded last chunk), all-gather of the spectra planes / W W^T partials /
    lin-quad -- factorises like the all-reduced unfused DP step: identical W on both
    ranks, pass counts +-1, errors of same-pass replicates to 1e-5.  The third case is a
    mixed-K batch (a cNMF K grid): one packed exchange per K group and step, issued in
    the background under the other group's compute.  Shapes large enough
    that both solves run the production cooperative slices (800 cells per rank and step,
    800 genes: S > 1 on both sides)."""
    X = normalized_counts_matrix(3200, 800, n_programs=6, seed=9)
    seeds = list(range(31, 31 + R))
    kw = dict(online_chunk_size=1600, online_max_pass=12)
    for fused in ("1", "0"):
        _spawn(W.dp_fused_worker, 2, X, K, seeds, kw, str(tmp_path), fused, timeout=150)
    # the packed step with its reduce-scatter / all-gather as one-shot xGMI kernels
    _spawn(W.dp_fused_worker, 2, X, K, seeds, kw, str(tmp_path), "1", "xgmi", timeout=150)
    for r in range(2):
        assert bool(np.load(tmp_path / f"dpf1_{r}.npz.npy")[0])
        assert not bool(np.load(tmp_path / f"dpf0_{r}.npz.npy")[0])
        # the cooperative-slice solves ran multi-process (both sides sliced)
        S_h, S_w, units = np.load(tmp_path / f"dpfS1_{r}.npy")
        assert S_h > 1 and S_w > 1, (S_h, S_w)
        # the mixed-K batch: two exchange units per step (its K groups), each one's
        # collectives issued in the background under the other's compute
        assert units == (2 if isinstance(K, tuple) else 1)
        took, used = np.load(tmp_path / f"dpf1x_{r}.npz.npy")
        assert bool(took) and bool(used)
    Wf = np.load(tmp_path / "dpfW1_0.npy")
    np.testing.assert_array_equal(Wf, np.load(tmp_path / "dpfW1_1.npy"))
    # 2 ranks: gloo's and the kernels' sums are the same float32 a + b -- bitwise
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"dpfW1x_{r}.npy"), Wf)
        np.testing.assert_array_equal(np.load(tmp_path / f"dpferr1x_{r}.npy"),
                                      np.load(tmp_path / "dpferr1_0.npy"))
    ef, eu = np.load(tmp_path / "dpferr1_0.npy"), np.load(tmp_path / "dpferr0_0.npy")
    itf, itu = np.load(tmp_path / "dpfit1_0.npy"), np.load(tmp_path / "dpfit0_0.npy")
    assert np.abs(itf - itu).max() <= 1
    same = itf == itu
    assert same.mean() > 0.6
    np.testing.assert_allclose(ef[same], eu[same], rtol=1e-5)

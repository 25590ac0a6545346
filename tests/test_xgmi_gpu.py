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
    _spawn(W.xgmi_worker, 2, str(tmp_path))
    r0, r1 = (np.load(tmp_path / f"xgmi{r}.npz") for r in range(2))
    n_calls = sum(1 for k in r0.files if k.startswith("err"))
    assert n_calls == 61
    for i in range(n_calls):
        assert r0[f"err{i}"] == 0.0 and r1[f"err{i}"] == 0.0, i
        np.testing.assert_array_equal(r0[f"sum{i}"], r1[f"sum{i}"])   # identical on ranks
    for r in (r0, r1):
        assert bool(r["comm_is_xgmi"])
        np.testing.assert_array_equal(r["comm"], np.full(10, 3.0, dtype=np.float32))
    assert bool(r0["timed_out"]) and not bool(r1["timed_out"])
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
        _spawn(W.xgmi_dp_worker, 2, X, K, seeds, kw, str(tmp_path), ar)
    assert bool(np.load(tmp_path / "used_xgmi0.npy"))
    assert not bool(np.load(tmp_path / "used_rccl0.npy"))
    Wx, Wg = np.load(tmp_path / "W_xgmi0.npy"), np.load(tmp_path / "W_rccl0.npy")
    np.testing.assert_array_equal(Wx, np.load(tmp_path / "W_xgmi1.npy"))
    np.testing.assert_allclose(Wx, Wg, rtol=1e-4, atol=1e-6)
    ref = NMFBatchSolver(torch.from_numpy(X).cuda(), NMFOptions(n_components=K, **kw)).run(seeds)
    np.testing.assert_allclose(np.load(tmp_path / "err_xgmi0.npy"), ref.err, rtol=1e-3)

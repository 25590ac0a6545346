"""Block-principal-pivoting NNLS (models/bpp.py; nmf-torch ``algo='bpp'``)
against scipy.optimize.nnls and the KKT conditions, and ANLS-BPP NMF in the engine."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
from scipy.optimize import nnls

from cnmf_torch_amd.models.bpp import nnls_bpp
from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions, run_nmf_batch


def _ls_problem(R=3, m=40, K=7, n=25, seed=0):
    rs = np.random.default_rng(seed)
    A = rs.random((R, m, K))
    Y = rs.random((R, m, n)) - 0.3
    G = np.einsum("rmk,rml->rkl", A, A)
    B = np.einsum("rmk,rmn->rkn", A, Y)
    return A, Y, G, B


def test_matches_scipy_nnls():
    A, Y, G, B = _ls_problem()
    X = nnls_bpp(torch.from_numpy(G), torch.from_numpy(B)).numpy()
    for r in range(A.shape[0]):
        for j in range(Y.shape[2]):
            ref, _ = nnls(A[r], Y[r, :, j])
            np.testing.assert_allclose(X[r, :, j], ref, rtol=1e-6, atol=1e-9)


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 10_000), K=st.integers(1, 16), n=st.integers(1, 40),
       l1=st.sampled_from([0.0, 0.3]), l2=st.sampled_from([0.0, 0.5]))
def test_kkt_point(seed, K, n, l1, l2):
    g = torch.Generator().manual_seed(seed)
    A = torch.rand((2, K + 3, K), generator=g, dtype=torch.float64)
    G = A.transpose(1, 2) @ A
    B = torch.randn((2, K, n), generator=g, dtype=torch.float64)
    X = nnls_bpp(G, B, l1=l1, l2=l2)
    assert torch.all(X >= 0)
    grad = (G + l2 * torch.eye(K, dtype=torch.float64)) @ X - (B - l1)
    pg = torch.where(X > 0, grad, torch.clamp(grad, max=0.0))   # projected gradient
    assert pg.abs().max().item() < 1e-8 * (B.abs().max().item() + 1.0)


def test_rank_deficient_gram_reaches_nnls_optimum():
    A, Y, _, _ = _ls_problem(R=1, K=5, seed=2)
    A = np.concatenate([A, A[:, :, :1]], axis=2)                 # duplicated column
    G = np.einsum("rmk,rml->rkl", A, A)
    B = np.einsum("rmk,rmn->rkn", A, Y)
    X = nnls_bpp(torch.from_numpy(G), torch.from_numpy(B)).numpy()
    for j in range(Y.shape[2]):
        ref, rnorm = nnls(A[0], Y[0, :, j])
        got = np.linalg.norm(A[0] @ X[0, :, j] - Y[0, :, j])
        assert got <= rnorm * (1 + 1e-7) + 1e-10


def _low_rank(seed=0, n=120, g=60, k=4):
    rs = np.random.default_rng(seed)
    return torch.from_numpy(rs.gamma(1.0, 1.0, (n, k)) @ rs.gamma(1.0, 1.0, (k, g))
                            + 0.05 * rs.random((n, g)))


def test_anls_bpp_batch_is_monotone_and_beats_mu():
    X = _low_rank()
    errs = {}
    for algo in ("bpp", "mu"):
        errs[algo] = []
        for it in (1, 2, 4, 8):
            opts = NMFOptions(n_components=4, mode="batch", algo=algo, batch_max_iter=it,
                              tol=-1.0, fp_precision="double", loss_every=1)
            errs[algo].append(float(NMFBatchSolver(X, opts).run([7]).err[0]))
    e = errs["bpp"]
    assert all(b <= a * (1 + 1e-10) for a, b in zip(e, e[1:])), e
    assert errs["bpp"][-1] < errs["mu"][-1]


def test_online_bpp_factorisation():
    X = _low_rank(seed=1, n=300).float().numpy()
    res = run_nmf_batch(X, 4, [1, 2, 3], algo="bpp", online_chunk_size=100, online_max_pass=8)
    assert np.all(np.isfinite(res.err))
    W = res.W.cpu().numpy()
    assert W.shape == (12, X.shape[1]) and np.all(W >= 0)
    mu = run_nmf_batch(X, 4, [1, 2, 3], algo="mu", online_chunk_size=100, online_max_pass=8)
    assert np.all(res.err <= mu.err * 1.05)


def test_bpp_rejects_beta_losses():
    with pytest.raises(ValueError):
        NMFOptions(n_components=3, algo="bpp", beta_loss="kullback-leibler").validate()


@pytest.mark.gpu
def test_bpp_on_gpu_matches_cpu():
    _, _, G, B = _ls_problem(R=4, K=10, n=300, seed=5)
    Gt, Bt = torch.from_numpy(G), torch.from_numpy(B)
    cpu = nnls_bpp(Gt, Bt)
    gpu = nnls_bpp(Gt.cuda(), Bt.cuda()).cpu()
    torch.testing.assert_close(gpu, cpu, rtol=1e-9, atol=1e-11)
    X = _low_rank(seed=3, n=2000, g=300).float().numpy()
    res = run_nmf_batch(X, 6, [11, 12], algo="bpp", device="cuda", online_chunk_size=700,
                        online_max_pass=5)
    assert np.all(np.isfinite(res.err)) and np.all(res.W.cpu().numpy() >= 0)

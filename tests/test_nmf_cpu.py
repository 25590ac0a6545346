"""CPU numerics of the replicate-batched NMF engine (models/nmf.py) against scikit-learn.

sklearn's ``non_negative_factorization(solver='mu')`` is the reference math the SURVEY
points at for the beta-divergence updates (sklearn/decomposition/_nmf.py:526-728); with
``init='custom'`` and the same starting factors, the batch MU trajectory must agree.
"""
import numpy as np
import pytest
import torch
from sklearn.decomposition import non_negative_factorization

from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions, run_nmf
from cnmf_torch_amd.ops import reference
from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

EPS32 = float(np.finfo(np.float32).eps)


def _data(n=240, g=90, seed=0):
    X = normalized_counts_matrix(n, g, n_programs=4, seed=seed).astype(np.float64)
    return X + 0.01  # strictly positive: sklearn zeroes sub-eps factors for beta <= 1


@pytest.mark.parametrize("beta_loss,beta", [("kullback-leibler", 1.0), ("itakura-saito", 0.0),
                                            (1.5, 1.5)])
def test_batch_beta_mu_matches_sklearn(beta_loss, beta):
    X = _data()
    K, n_it = 4, 25
    rng = np.random.default_rng(3)
    H0 = rng.random((X.shape[0], K)) + 0.1      # usages  (sklearn W)
    W0 = rng.random((K, X.shape[1])) + 0.1      # spectra (sklearn H)
    Wsk, Hsk, _ = non_negative_factorization(X, W=H0.copy(), H=W0.copy(), n_components=K,
                                             init="custom", solver="mu", beta_loss=beta_loss,
                                             max_iter=n_it, tol=0.0)
    opts = NMFOptions(n_components=K, beta_loss=beta_loss, mode="batch", batch_max_iter=n_it,
                      tol=-1.0, fp_precision="double", eps=EPS32, loss_every=5)
    res = NMFBatchSolver(torch.from_numpy(X), opts).run(
        [1], HT0=torch.from_numpy(H0.T.copy()), W0=torch.from_numpy(W0))
    np.testing.assert_allclose(res.usages(0).numpy(), Wsk, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(res.spectra(0).numpy(), Hsk, rtol=1e-7, atol=1e-9)
    # reported error = sqrt(2 * D_beta) of the final factors
    P = Wsk @ Hsk
    D = float(reference.beta_loss_terms(torch.from_numpy(X), torch.from_numpy(P), beta,
                                        EPS32).sum())
    assert abs(res.err[0] - np.sqrt(2 * D)) <= 1e-9 * max(1.0, np.sqrt(2 * D))


def test_beta_contract_reference_identities():
    """side 'h'/'w' numerators are the two contractions of Q = X / (HT^T W)."""
    g = torch.Generator().manual_seed(0)
    R, K, N, G = 2, 3, 50, 40
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.1
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.1
    nh, dh, loss = reference.beta_contract(0, X, HT, W, 1.0, 1e-12, True, True)
    nw, dw, _ = reference.beta_contract(1, X, HT, W, 1.0, 1e-12, True, False)
    assert dh is None and dw is None
    for r in range(R):
        Q = X / (HT[r].t() @ W[r])
        torch.testing.assert_close(nh[r], W[r] @ Q.t())
        torch.testing.assert_close(nw[r], HT[r] @ Q)
        P = HT[r].t() @ W[r]
        kl = (X * torch.log(X / P) - X + P).sum()
        torch.testing.assert_close(loss[r], kl)


@pytest.mark.parametrize("mode", ["online", "batch"])
def test_kl_decreases_and_recovers(mode):
    X = _data(400, 120, seed=2)
    H, W, err = run_nmf(X, 4, beta_loss="kullback-leibler", mode=mode, random_state=5,
                        online_chunk_size=150, batch_max_iter=200, tol=1e-5)
    assert H.shape == (400, 4) and W.shape == (4, 120)
    assert np.all(H >= 0) and np.all(W >= 0)
    # the error must be well below that of the random init and below a rank-1 model
    P1 = np.outer(X.sum(1), X.sum(0)) / X.sum()
    kl1 = float(reference.beta_loss_terms(torch.from_numpy(X), torch.from_numpy(P1), 1.0,
                                          1e-16).sum())
    assert err < 0.8 * np.sqrt(2 * kl1), (err, np.sqrt(2 * kl1))


def test_online_kl_passes_monotone_errors():
    X = _data(300, 80, seed=4)
    opts = NMFOptions(n_components=3, beta_loss="kullback-leibler", mode="online",
                      online_chunk_size=100, online_max_pass=6, tol=-1.0, fp_precision="double")
    solver = NMFBatchSolver(torch.from_numpy(X), opts)
    errs = []
    for p in (1, 2, 4, 6):
        solver.opts.online_max_pass = p
        errs.append(float(solver.run([7]).err[0]))
    assert all(b <= a * (1 + 1e-9) for a, b in zip(errs, errs[1:])), errs


def test_pass_counts_and_convergence_flags():
    X = _data(200, 60, seed=6).astype(np.float32)
    opts = NMFOptions(n_components=3, online_chunk_size=80, online_max_pass=7, tol=1e-3)
    res = NMFBatchSolver(torch.from_numpy(X), opts).run([1, 2, 3])
    assert ((res.n_iter >= 1) & (res.n_iter <= 7)).all(), res.n_iter
    # a replicate that did not converge ran every pass
    assert all(c or n == 7 for c, n in zip(res.converged, res.n_iter))


@pytest.mark.parametrize("variant", ["nndsvd", "nndsvda"])
def test_nndsvd_init_matches_sklearn(variant):
    from sklearn.decomposition._nmf import _initialize_nmf

    from cnmf_torch_amd.models.nmf import _nndsvd
    from cnmf_torch_amd.parallel.comm import LocalComm

    X = _data(150, 70, seed=8)
    K = 4
    Wsk, Hsk = _initialize_nmf(X, K, init=variant, random_state=0)
    H, W = _nndsvd(torch.from_numpy(X), K, variant, LocalComm())
    # randomized vs exact SVD: agree to the randomized solver's accuracy
    np.testing.assert_allclose(H.numpy(), Wsk, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(W.numpy(), Hsk, rtol=1e-5, atol=1e-6)


def test_halsvar_inner_loops_and_online_equivalence():
    """'halsvar' (batch): HALS half-steps iterated to batch_hals_tol reach a lower error
    per outer iteration than one-sweep 'hals'; online, both are the same chunk solves."""
    X = torch.from_numpy(normalized_counts_matrix(300, 120, 5, seed=21))
    errs = {}
    for algo in ("hals", "halsvar"):
        _, _, errs[algo] = run_nmf(X, 5, algo=algo, mode="batch", batch_max_iter=5, tol=-1.0,
                                   random_state=3)
    assert errs["halsvar"] < errs["hals"]
    on = {a: run_nmf(X, 5, algo=a, mode="online", online_chunk_size=100, online_max_pass=4,
                     random_state=3) for a in ("hals", "halsvar")}
    for x, y in zip(on["hals"], on["halsvar"]):
        np.testing.assert_array_equal(x, y)
    with pytest.raises(ValueError):
        NMFOptions(n_components=3, algo="halsvar", beta_loss="kullback-leibler").validate()


@pytest.mark.parametrize("beta_loss", ["kullback-leibler", "itakura-saito"])
def test_online_beta_converges_close_to_batch(beta_loss):
    """Online beta-MU (the mode the reference CLI hard-codes, cnmf.py:765, for every
    --beta-loss, cnmf.py:1426) must converge like the Frobenius path: converged=True in
    fewer than online_max_pass passes, final error within 1 % of batch MU."""
    X = normalized_counts_matrix(3000, 400, n_programs=6, seed=0)
    kw = dict(beta_loss=beta_loss, online_chunk_size=1000, online_chunk_max_iter=1000,
              batch_max_iter=2000)
    on = NMFBatchSolver(torch.from_numpy(X), NMFOptions(n_components=6, mode="online", **kw)).run([1, 2])
    ba = NMFBatchSolver(torch.from_numpy(X), NMFOptions(n_components=6, mode="batch", **kw)).run([1, 2])
    assert on.converged.all(), (on.n_iter, on.err)
    assert (on.n_iter < 20).all(), on.n_iter
    assert (np.abs(on.err - ba.err) / ba.err < 0.01).all(), (on.err, ba.err)
    # the usage loop ran several steps per chunk (block-objective rule), not ~1
    assert min(on.stats["h_inner_iters"]) >= 5 * 3 * min(on.n_iter)


@pytest.mark.parametrize("beta,gamma", [(1.0, 1.0), (0.0, 0.5), (1.5, 1.0)])
def test_beta_w_update_single_chunk_is_sklearn_mu_step(beta, gamma):
    """With no earlier chunk statistics the anchored online spectra step is exactly one
    multiplicative update W <- W (num/den)^gamma (sklearn _nmf.py:526-728)."""
    g = torch.Generator().manual_seed(2)
    R, K, N, G = 2, 3, 60, 40
    X = torch.rand((N, G), generator=g, dtype=torch.float64) + 0.05
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.1
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.1
    num, den, _ = reference.beta_contract(1, X, HT, W, beta, 1e-16, True, False)
    if den is None:
        den = HT.sum(dim=2, keepdim=True).expand_as(num)
    expect = W * (num / den) ** gamma
    Wc = W.clone()
    kl = beta == 1.0
    An = torch.zeros_like(W)
    Ad = torch.zeros((R, K), dtype=W.dtype) if kl else torch.zeros_like(W)
    an = torch.zeros_like(W)
    dn = None if kl else torch.zeros_like(W)
    nW, dW, _ = reference.beta_contract(1, X, HT, W, beta, 1e-16, True, False)
    act = torch.ones(R, dtype=torch.int32)
    it = torch.zeros(R, dtype=torch.int32)
    reference.beta_w_update(Wc, nW.unsqueeze(0), None if kl else dW.unsqueeze(0),
                            HT.sum(dim=2) if kl else None, An, Ad, an, dn, beta, gamma, 0.0,
                            0.0, 1e-16, 1e-12, act, it)
    torch.testing.assert_close(Wc, expect)
    torch.testing.assert_close(an, W ** (1.0 / gamma) * num)
    assert it.tolist() == [1, 1]


def test_beta_h_loss_rule_checks_every_n_steps():
    """conv_mode 1 of the fused usage step: the objective is recorded every check_every
    steps and a replicate stops only at a check (never from the iterate change)."""
    g = torch.Generator().manual_seed(4)
    R, K, N, G = 3, 4, 80, 50
    X = torch.rand((N, G), generator=g, dtype=torch.float64) + 0.05
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.1
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.1
    act = torch.ones(R, dtype=torch.int32)
    it = torch.zeros(R, dtype=torch.int32)
    hs = torch.zeros((R, 2), dtype=torch.float64)
    stopped_at = {}
    for step in range(60):
        reference.beta_update_h(X, HT, W, 1.0, 1e-16, act=act, tol=0.05, iters=it,
                                conv_mode=1, check_every=5, hstate=hs)
        for r in range(R):
            if act[r] == 0 and r not in stopped_at:
                stopped_at[r] = step
        if act.sum() == 0:
            break
    assert stopped_at, "loose tolerance must stop"
    assert all(s % 5 == 0 and s >= 5 for s in stopped_at.values()), stopped_at


@pytest.mark.parametrize("mode,algo", [("online", "mu"), ("online", "hals"), ("batch", "mu"),
                                       ("online", "bpp")])
def test_mixed_k_ragged_batch_matches_single_k_runs(mode, algo):
    """The whole K x n_iter grid in ONE ragged batch (one pass loop, one data-side GEMM per
    chunk for every K) gives every replicate exactly its single-K run: same passes, same
    convergence flags, same factors up to fp64 summation order."""
    X = torch.from_numpy(_data(300, 80, seed=2))
    kw = dict(mode=mode, algo=algo, online_chunk_size=110, online_max_pass=6,
              batch_max_iter=40, fp_precision="double")
    ks = [3, 5, 3, 4, 5, 4, 3]
    seeds = [11, 12, 13, 14, 15, 16, 17]
    solver = NMFBatchSolver(X, NMFOptions(n_components=3, **kw))
    mixed = solver.run(seeds, ks=ks)
    assert mixed.K is None and list(mixed.ks) == ks
    for K in sorted(set(ks)):
        idx = [i for i, k in enumerate(ks) if k == K]
        ref = NMFBatchSolver(X, NMFOptions(n_components=K, **kw)).run([seeds[i] for i in idx])
        for j, i in enumerate(idx):
            assert mixed.n_iter[i] == ref.n_iter[j]
            assert mixed.converged[i] == ref.converged[j]
            np.testing.assert_allclose(mixed.err[i], ref.err[j], rtol=1e-9)
            np.testing.assert_allclose(mixed.spectra(i).numpy(), ref.spectra(j).numpy(),
                                       rtol=1e-7, atol=1e-10)
            np.testing.assert_allclose(mixed.usages(i).numpy(), ref.usages(j).numpy(),
                                       rtol=1e-7, atol=1e-10)


def test_mixed_k_beta_request_splits_by_k():
    X = torch.from_numpy(_data(200, 60, seed=4))
    kw = dict(beta_loss="kullback-leibler", online_chunk_size=100, online_max_pass=3,
              fp_precision="double")
    solver = NMFBatchSolver(X, NMFOptions(n_components=2, **kw))
    res = solver.run([5, 6, 7], ks=[4, 2, 4])
    ref4 = NMFBatchSolver(X, NMFOptions(n_components=4, **kw)).run([5, 7])
    np.testing.assert_allclose(res.spectra(2).numpy(), ref4.spectra(1).numpy(), rtol=1e-9)
    assert res.spectra(1).shape == (2, 60)


def test_planes_only_x_factorises_like_the_resident_matrix():
    """A matrix held only as split-GEMM planes, built block by block (nmf.PlanesOnlyX over
    nmf.RowBlocks: the route for 10M x 5k on one GPU, where fp32 X and its planes do not
    fit together) factorises like the resident fp32 matrix: same pass counts, errors to
    fp32 rounding.  Count detection runs per block; reads of X raise."""
    import torch

    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions, PlanesOnlyX, RowBlocks
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(640, 96, n_programs=4, seed=2))
    opts = NMFOptions(n_components=4, online_chunk_size=160, online_max_pass=6)
    src = RowBlocks(640, 96, lambda: ((a, X[a:a + 98]) for a in range(0, 640, 98)), "cpu")
    with pytest.raises(ValueError, match="multiple of 4"):
        PlanesOnlyX(src)
    src = RowBlocks(640, 96, lambda: ((a, X[a:a + 128]) for a in range(0, 640, 128)), "cpu")
    px = PlanesOnlyX(src)
    assert px.planes.unit is not None and px.planes.pb in (1, 2)   # exact count planes
    ref = NMFBatchSolver(X, opts).run([5, 6, 7])
    got = NMFBatchSolver(px, opts).run([5, 6, 7])
    np.testing.assert_array_equal(got.n_iter, ref.n_iter)
    np.testing.assert_allclose(got.err, ref.err, rtol=1e-5)
    with pytest.raises(ValueError, match="PlanesOnlyX supports"):
        NMFBatchSolver(px, NMFOptions(n_components=4, mode="batch"))


def test_native_rank_padding_rule():
    """GPU rank padding (models.nmf.native_rank): K <= 32 as is, multiples of 8 up to 64,
    multiples of 16 up to 128 (the matrix-core wide MU solve), K itself beyond (the
    rank-general solve, solve_any.hip)."""
    from cnmf_torch_amd.models.nmf import kernel_max_rank, native_rank

    assert [native_rank(k) for k in (1, 10, 32)] == [1, 10, 32]
    assert [native_rank(k) for k in (33, 40, 41, 64)] == [40, 40, 48, 64]
    assert [native_rank(k) for k in (65, 80, 81, 100, 128)] == [80, 80, 96, 112, 128]
    assert [native_rank(k) for k in (129, 200, 1000)] == [129, 200, 1000]
    assert kernel_max_rank(2.0, "mu") is None and kernel_max_rank(2.0, "hals") == 512
    assert kernel_max_rank(1.0, "mu") is None and kernel_max_rank(0.0, "mu") is None


def test_padded_rank_solve_equals_unpadded_on_cpu():
    """The padding argument itself: zero components appended to x, numer and the Gram stay
    zero under MU and leave the true components' iterates unchanged (CPU reference op)."""
    import torch

    from cnmf_torch_amd import ops

    g = torch.Generator().manual_seed(3)
    K, Kp, n = 70, 80, 300
    Wf = torch.rand((K, 50), generator=g, dtype=torch.float64)
    gram = Wf @ Wf.t()
    numer = gram @ torch.rand((K, n), generator=g, dtype=torch.float64)
    x0 = torch.rand((K, n), generator=g, dtype=torch.float64) + 0.1
    x = x0.clone()[None]
    ops.solve("mu", x, numer[None], gram[None], max_iter=25, tol=0.0)
    xp = torch.zeros((1, Kp, n), dtype=torch.float64)
    npd = torch.zeros((1, Kp, n), dtype=torch.float64)
    gp = torch.zeros((1, Kp, Kp), dtype=torch.float64)
    xp[0, :K], npd[0, :K], gp[0, :K, :K] = x0, numer, gram
    ops.solve("mu", xp, npd, gp, max_iter=25, tol=0.0)
    assert torch.equal(xp[0, K:], torch.zeros((Kp - K, n), dtype=torch.float64))
    torch.testing.assert_close(xp[0, :K], x[0], rtol=1e-12, atol=0)

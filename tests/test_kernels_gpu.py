"""HIP kernel numerics vs the PyTorch reference (fp32 on CPU, and fp64 oracle).

Every test here runs the native gfx950 kernels; they fail (not skip) on a GPU box if
the extension did not load.
"""
import os

import numpy as np
import pytest
import torch

from cnmf_torch_amd import ops
from cnmf_torch_amd.ops import reference
from cnmf_torch_amd.utils.rng import philox_matrix

pytestmark = pytest.mark.gpu


def _problem(R, K, n, seed=0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    W = torch.rand((R, K, 64), generator=g, dtype=torch.float64) + 0.05
    gram = torch.bmm(W, W.transpose(1, 2))
    x_true = torch.rand((R, K, n), generator=g, dtype=torch.float64)
    numer = torch.bmm(gram, x_true) * (1 + 0.05 * torch.rand((R, K, n), generator=g, dtype=torch.float64))
    x0 = torch.rand((R, K, n), generator=g, dtype=torch.float64) + 0.1
    return x0.to(dtype), numer.to(dtype), gram.to(dtype)


def test_native_extension_loaded():
    assert ops.native_available(), f"HIP extension failed to load: {ops.native_error()}"


@pytest.mark.parametrize("algo", ["mu", "hals"])
@pytest.mark.parametrize("K", [3, 10, 17, 32])
@pytest.mark.parametrize("conv_mode", [0, 1])
def test_solve_matches_reference(algo, K, conv_mode):
    R, n = 6, 3001
    x0, numer, gram = _problem(R, K, n, seed=K)
    dev = torch.device("cuda")
    # fixed iteration count (tol < 0) isolates the arithmetic from convergence decisions
    for max_iter, tol in ((7, -1.0), (200, 1e-3)):
        xg = x0.clone().to(dev)
        lin_g = torch.zeros(R, device=dev)
        quad_g = torch.zeros(R, device=dev)
        it_g = torch.zeros(R, dtype=torch.int32, device=dev)
        ops.solve(algo, xg, numer.to(dev), gram.to(dev), max_iter=max_iter, tol=tol,
                  lin_out=lin_g, quad_out=quad_g, iters_out=it_g, conv_mode=conv_mode,
                  check_every=5)
        xr = x0.clone().double()
        lin_r = torch.zeros(R, dtype=torch.float64)
        quad_r = torch.zeros(R, dtype=torch.float64)
        it_r = torch.zeros(R, dtype=torch.int32)
        reference.solve(ops.ALGOS[algo], xr, numer.double(), gram.double(), None, max_iter, tol,
                        0.0, 0.0, 0.0, 1e-16, lin_r, quad_r, it_r, 1, conv_mode, 5)
        torch.cuda.synchronize()
        if tol < 0:
            assert it_g.cpu().tolist() == [max_iter] * R
            torch.testing.assert_close(xg.cpu().double(), xr, rtol=2e-4, atol=1e-4)
        else:
            # convergence decisions may differ by a step at the boundary; compare solutions
            diff = (xg.cpu().double() - xr).norm() / xr.norm()
            assert diff < 5e-3, diff
        torch.testing.assert_close(lin_g.cpu().double(), lin_r, rtol=1e-3, atol=1e-3)
        torch.testing.assert_close(quad_g.cpu().double(), quad_r, rtol=1e-3, atol=1e-3)


def test_solve_strided_and_rep_index():
    R, K, N = 5, 7, 2000
    dev = torch.device("cuda")
    HT = torch.rand((R * K, N), device=dev) + 0.1
    numer = torch.rand((R * K, 600), device=dev)
    W = torch.rand((R, K, 40), device=dev)
    gram = torch.bmm(W, W.transpose(1, 2))
    ref = HT.clone().cpu()
    view = HT.view(R, K, N)[:, :, 300:900]
    rep = torch.tensor([0, 3], dtype=torch.int32, device=dev)
    ops.solve("mu", view, numer.view(R, K, 600), gram, rep_index=rep, max_iter=4)
    rview = ref.view(R, K, N)[:, :, 300:900]
    reference.solve(0, rview, numer.cpu().view(R, K, 600), gram.cpu(), rep.cpu(), 4, -1.0, 0, 0, 0,
                    1e-16, None, None, None)
    torch.cuda.synchronize()
    torch.testing.assert_close(HT.cpu(), ref, rtol=1e-4, atol=1e-6)
    # untouched replicates / columns really are untouched
    untouched = HT.view(R, K, N)[1]
    assert torch.equal(untouched.cpu(), ref.view(R, K, N)[1])


@pytest.mark.parametrize("algo", ["mu", "hals"])
@pytest.mark.parametrize("conv_mode", [0, 1])
def test_solve_coop_split_matches_single_workgroup(algo, conv_mode):
    """S workgroups per replicate (cross-WG reductions) == one workgroup per replicate."""
    R, K, n = 5, 10, 9001
    x0, numer, gram = _problem(R, K, n, seed=3)
    dev = torch.device("cuda")
    numer, gram = numer.to(dev), gram.to(dev)
    outs = {}
    for S in (1, 2, 3, 7):
        for max_iter, tol in ((9, -1.0), (300, 1e-4)):
            xg = x0.clone().to(dev)
            lin = torch.zeros(R, device=dev)
            quad = torch.zeros(R, device=dev)
            it = torch.zeros(R, dtype=torch.int32, device=dev)
            ops.solve(algo, xg, numer, gram, max_iter=max_iter, tol=tol, lin_out=lin,
                      quad_out=quad, iters_out=it, conv_mode=conv_mode, check_every=5, coop=S)
            outs[(S, tol)] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu())
    ops.coop_check(dev)
    for S in (2, 3, 7):
        for tol in (-1.0, 1e-4):
            x1, l1, q1, i1 = outs[(1, tol)]
            xs, ls, qs, is_ = outs[(S, tol)]
            if tol < 0:
                assert torch.equal(xs, x1)          # column updates are independent of S
                assert is_.tolist() == [9] * R
            else:
                assert (is_ - i1).abs().max() <= 5
                assert ((xs - x1).norm() / x1.norm()) < 2e-3
            torch.testing.assert_close(ls, l1, rtol=1e-4, atol=1e-3)
            torch.testing.assert_close(qs, q1, rtol=1e-4, atol=1e-3)


def test_solve_coop_with_active_mask_and_rep_index():
    R, K, n = 8, 7, 5000
    x0, numer, gram = _problem(R, K, n, seed=5)
    dev = torch.device("cuda")
    active = torch.tensor([1, 0, 1, 1, 0, 1, 1, 1], dtype=torch.int32, device=dev)
    ri = torch.tensor([0, 1, 2, 5, 7], dtype=torch.int32, device=dev)
    res = []
    for S in (1, 4):
        xg = x0.clone().to(dev)
        ops.solve("mu", xg, numer.to(dev), gram.to(dev), rep_index=ri, max_iter=50, tol=1e-5,
                  conv_mode=1, check_every=5, active=active, coop=S)
        res.append(xg.cpu())
    ops.coop_check(dev)
    untouched = [1, 3, 4, 6]
    for r in untouched:
        assert torch.equal(res[1][r], x0[r])
    torch.testing.assert_close(res[1], res[0], rtol=2e-3, atol=1e-4)


def test_solve_split_columns():
    R, K, n = 4, 9, 50000
    x0, numer, gram = _problem(R, K, n, seed=3)
    dev = torch.device("cuda")
    xg = x0.clone().to(dev)
    lin = torch.zeros(R, device=dev)
    quad = torch.zeros(R, device=dev)
    ops.solve("mu", xg, numer.to(dev), gram.to(dev), max_iter=1, nsplit=7, lin_out=lin,
              quad_out=quad)
    xr = x0.clone().double()
    lr = torch.zeros(R, dtype=torch.float64)
    qr = torch.zeros(R, dtype=torch.float64)
    reference.solve(0, xr, numer.double(), gram.double(), None, 1, -1.0, 0, 0, 0, 1e-16, lr, qr,
                    None)
    torch.cuda.synchronize()
    torch.testing.assert_close(xg.cpu().double(), xr, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(lin.cpu().double(), lr, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("mode", [0, 1])
def test_philox_matches_numpy(mode):
    dev = torch.device("cuda")
    R, rows, cols = 3, 1001, 7
    seeds = torch.tensor([1, 123456789, 2**31 - 2], dtype=torch.int64)
    scales = torch.tensor([1.0, 0.5, 2.0])
    out = torch.empty((R, rows, cols), device=dev)
    ops.philox_fill(out, seeds, scales, 5, mode)
    torch.cuda.synchronize()
    for r in range(R):
        ref = philox_matrix(int(seeds[r]), 5, rows, cols, mode) * float(scales[r])
        np.testing.assert_allclose(out[r].cpu().numpy(), ref, rtol=2e-6, atol=1e-7)
    # transposed layout + row offset (cell-sharded init)
    HT = torch.empty((R * cols, 333), device=dev)
    ops.philox_fill(HT.as_strided((R, 333, cols), (cols * 333, 1, 333)), seeds, scales, 5, mode,
                    row_offset=17)
    torch.cuda.synchronize()
    for r in range(R):
        ref = philox_matrix(int(seeds[r]), 5, 333, cols, mode, row_offset=17) * float(scales[r])
        np.testing.assert_allclose(HT[r * cols:(r + 1) * cols].t().cpu().numpy(), ref, rtol=2e-6,
                                   atol=1e-7)


@pytest.mark.parametrize("algo,beta_loss", [("mu", "frobenius"), ("hals", "frobenius"),
                                            ("halsvar", "frobenius"), ("mu", "kullback-leibler")])
@pytest.mark.parametrize("mode", ["online", "batch"])
def test_nmf_batch_gpu_matches_cpu(algo, mode, beta_loss):
    from cnmf_torch_amd.models.nmf import run_nmf_batch

    rs = np.random.default_rng(0)
    N, G, K = 1500, 400, 6
    X = (rs.gamma(1, 1, (N, K)) @ rs.gamma(0.5, 1, (K, G)) + 0.1 * rs.random((N, G))).astype(
        np.float32)
    kw = dict(algo=algo, mode=mode, online_chunk_size=700, online_max_pass=5, batch_max_iter=40,
              beta_loss=beta_loss)
    g = run_nmf_batch(X, K, [11, 12, 13], device="cuda", **kw)
    c = run_nmf_batch(X, K, [11, 12, 13], device="cpu", **kw)
    # same init, same algorithm: errors agree to fp32 reassociation noise -- 1e-3 for
    # Frobenius MU (replicates that stopped at the same pass; the split-precision GEMMs
    # and MFMA solves only reorder fp32 sums); 3e-3 for HALS, whose coordinate-by-
    # coordinate sweeps carry a reordering into every later coordinate (batch HALS after 40
    # unconverged iterations measured 2.1e-3 on one replicate, 5e-10 on another); looser
    # for KL (its MU step divides by the reconstruction element-wise)
    assert np.abs(g.n_iter - c.n_iter).max() <= 1, (g.n_iter, c.n_iter)
    same = g.n_iter == c.n_iter
    assert same.sum() >= 2, (g.n_iter, c.n_iter)
    rel = np.abs(g.err - c.err) / np.abs(c.err)
    tol = 2e-2 if beta_loss != "frobenius" else (1e-3 if algo == "mu" else 3e-3)
    assert rel[same].max() <= tol, (rel, g.n_iter, c.n_iter)
    assert rel.max() <= 2e-2, rel
    Wg, Wc = g.W.cpu().numpy(), c.W.cpu().numpy()
    cos = (Wg * Wc).sum(1) / (np.linalg.norm(Wg, axis=1) * np.linalg.norm(Wc, axis=1) + 1e-30)
    assert np.median(cos) > 0.99, np.sort(cos)[:5]


@pytest.mark.parametrize("beta", [1.0, 0.0, 1.5])
@pytest.mark.parametrize("K", [3, 10, 17, 32, 40, 64])
def test_beta_contract_matches_reference(beta, K):
    """Fused MFMA beta-MU contraction (beta_mu.hip) vs a float64 PyTorch reference."""
    g = torch.Generator().manual_seed(K)
    R, N, G = 3, 1000 + 37, 300 + 5          # ragged vs the 64-wide strips / 256 chunks
    X = torch.rand((N + 3, G), generator=g, dtype=torch.float64)
    X[X < 0.3] = 0.0                          # zeros exercise the KL x>0 branch
    HT = torch.rand((R * K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R * K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    Xs = X[2:N + 2]                           # row-offset view (unaligned base pointer)
    active = torch.tensor([1, 0, 1], dtype=torch.int32)
    eps = 1e-10
    for side in ("h", "w"):
        ref = reference.beta_contract(0 if side == "h" else 1, Xs, HT.view(R, K, N),
                                      W.view(R, K, G), beta, eps, True, side == "h")
        out = ops.beta_contract(side, Xs.float().to(dev), HT.float().to(dev).view(R, K, N),
                                W.float().to(dev).view(R, K, G), beta, eps, True, side == "h",
                                active=active.to(dev))
        for r in (0, 2):
            torch.testing.assert_close(out[0][r].cpu().double(), ref[0][r], rtol=2e-4, atol=1e-4)
            if beta != 1.0:
                torch.testing.assert_close(out[1][r].cpu().double(), ref[1][r], rtol=2e-4,
                                           atol=1e-4)
            if side == "h":
                torch.testing.assert_close(out[2][r].cpu(), ref[2][r], rtol=1e-4, atol=1e-3)
        if beta == 1.0:
            assert out[1] is None
    # W-side split over cells == unsplit
    a = ops.beta_contract("w", X[:N].float().to(dev), HT.float().to(dev).view(R, K, N),
                          W.float().to(dev).view(R, K, G), beta, eps, splits=1)[0]
    b = ops.beta_contract("w", X[:N].float().to(dev), HT.float().to(dev).view(R, K, N),
                          W.float().to(dev).view(R, K, G), beta, eps, splits=5)[0]
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("beta", [1.0, 0.0])
def test_beta_update_h_fused_matches_reference(beta):
    """In-place fused usage update + on-device inner stopping rule == reference."""
    g = torch.Generator().manual_seed(1)
    R, K, N, G = 4, 10, 777, 260
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    act0 = torch.tensor([1, 1, 0, 1], dtype=torch.int32)
    # replicate 3 starts at its own fixed point-ish (tiny change) -> should stop
    ref_h = HT.clone()
    ref_act, ref_it = act0.clone(), torch.zeros(R, dtype=torch.int32)
    gpu_h = HT.float().to(dev)
    gpu_act, gpu_it = act0.to(dev), torch.zeros(R, dtype=torch.int32, device=dev)
    for _ in range(6):
        reference.beta_update_h(X, ref_h, W, beta, 1e-10, 0.01, 0.02, 1.0 if beta else 0.5,
                                ref_act, 0.02, ref_it)
        ops.beta_update_h(X.float().to(dev), gpu_h, W.float().to(dev), beta, 1e-10, 0.01, 0.02,
                          1.0 if beta else 0.5, gpu_act, 0.02, gpu_it)
    torch.testing.assert_close(gpu_h.cpu().double(), ref_h, rtol=1e-4, atol=1e-5)
    assert gpu_act.cpu().tolist() == ref_act.tolist()
    assert gpu_it.cpu().tolist() == ref_it.tolist()
    assert torch.equal(gpu_h[2].cpu(), HT[2].float())       # inactive replicate untouched
    # plain update (no act / tol): batch mode
    h1 = HT.float().to(dev)
    ops.beta_update_h(X.float().to(dev), h1, W.float().to(dev), beta, 1e-10)
    h2 = HT.clone()
    reference.beta_update_h(X, h2, W, beta, 1e-10)
    torch.testing.assert_close(h1.cpu().double(), h2, rtol=1e-4, atol=1e-5)


@pytest.fixture
def kl_fp16(monkeypatch):
    """The opt-in fp16-numerator KL kernels (CNMF_KL_FP16=1) for the duration of a test."""
    monkeypatch.setenv("CNMF_KL_FP16", "1")
    ops.refresh_env()
    assert ops.bp_mode(1.0) == ops.BP_KL_FP16
    yield
    monkeypatch.delenv("CNMF_KL_FP16")
    ops.refresh_env()


@pytest.mark.parametrize("beta", [1.0, 0.0, 1.5, "kl16"])
@pytest.mark.parametrize("K,N,G", [(3, 1037, 305), (10, 777, 320), (17, 300, 131),
                                   (32, 129, 64)])
def test_split_bf16_beta_kernels_match_fp64(beta, K, N, G, request):
    """beta_planes.hip (split-bf16 MFMA: 3-term num/den; P exact (6 terms) or KL's 3
    terms) vs the float64 reference: loss-only pass, W-side partials (float4 and scalar X
    paths: ragged G/N), and one fused usage step.  The default KL mode (kBpKLX: Q = X / P
    in two bf16 planes) is held to the same 5e-5 as IS / general beta -- the fp32
    accumulation bound of these sums.  "kl16" is the opt-in fp16 numerator
    (CNMF_KL_FP16=1: one fp16 plane of X / P, <= 2^-11 relative per term, random sign):
    5e-4 relative (129-term sums at K = 32)."""
    fp16 = beta == "kl16"
    if fp16:
        request.getfixturevalue("kl_fp16")
        beta = 1.0
    else:
        assert ops.bp_mode(beta) != ops.BP_KL_FP16
    g = torch.Generator().manual_seed(K + N)
    R = 3
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    X[X < 0.3] = 0.0
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    eps = 1e-10
    Xg, Hg, Wg = X.float().to(dev), HT.float().to(dev), W.float().to(dev)
    active = torch.tensor([1, 0, 1], dtype=torch.int32, device=dev)
    # loss
    kl = fp16
    ref_loss = reference.beta_contract(0, X, HT, W, beta, eps, False, True)[2]
    got = ops.beta_loss(Xg, Hg, Wg, beta, eps)
    torch.testing.assert_close(got.cpu(), ref_loss, rtol=1e-4 if beta == 1.0 else 2e-5,
                               atol=1e-6)
    # W-side partials, two split counts
    rn, rd, _ = reference.beta_contract(1, X, HT, W, beta, eps, True, False)
    XT = Xg.t().contiguous()
    for splits in (1, 3):
        num, den = ops.beta_w_partials(Xg, XT, Hg, Wg, beta, eps, active=active, splits=splits)
        for r in (0, 2):
            torch.testing.assert_close(num.sum(0)[r].cpu().double(), rn[r],
                                       rtol=5e-4 if kl else 5e-5, atol=1e-5)
            if beta != 1.0:
                torch.testing.assert_close(den.sum(0)[r].cpu().double(), rd[r], rtol=5e-5,
                                           atol=1e-5)
        assert (den is None) == (beta == 1.0)
    # one fused usage step, no rule: every replicate
    h1 = Hg.clone()
    ops.beta_h_block(Xg, h1, Wg, beta, eps, 1, gamma=1.0 if beta else 0.5)
    h2 = HT.clone()
    reference.beta_h_block(X, h2, W, beta, eps, 1, gamma=1.0 if beta else 0.5)
    torch.testing.assert_close(h1.cpu().double(), h2, rtol=5e-4 if kl else 5e-5, atol=1e-6)


@pytest.mark.parametrize("beta,K,N,G", [(1.0, 40, 300, 131), (1.0, 48, 257, 200),
                                        (1.0, 56, 200, 100), (1.0, 64, 129, 64),
                                        ("kl16", 48, 257, 200), ("kl16", 64, 129, 64),
                                        (0.0, 40, 300, 131), (1.5, 48, 257, 200),
                                        (0.0, 56, 200, 100)])
def test_split_bf16_beta_kernels_wide_k_match_fp64(beta, K, N, G, request):
    """The K > 32 instantiations of beta_planes (beta_planes_wide*.hip: KL (both numerator
    modes) to 64, IS / general beta to 56; one column tile per wave, one wave per SIMD)
    against the float64 reference: loss, W-side partials and one fused usage step, with
    the K <= 32 test's tolerances."""
    test_split_bf16_beta_kernels_match_fp64(beta, K, N, G, request)


@pytest.mark.parametrize("beta_loss", ["kullback-leibler", "itakura-saito"])
def test_online_beta_wide_k_runs_native_and_matches_cpu(beta_loss):
    """Online KL at K = 48 (IS at K = 40) runs on the native kernels -- padded to a
    multiple of 8, no eager-PyTorch routing warning -- and factorises like the CPU
    engine from the same seeds: objectives within 2e-3, passes within 2."""
    import warnings

    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    K = 48 if beta_loss == "kullback-leibler" else 40
    Xn = normalized_counts_matrix(1200, 300, n_programs=8, seed=3)
    opts = NMFOptions(n_components=K, beta_loss=beta_loss, online_chunk_size=600,
                      online_chunk_max_iter=200, online_max_pass=6)
    seeds = [5, 6, 7]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        g = NMFBatchSolver(torch.from_numpy(Xn).cuda(), opts).run(seeds)
    c = NMFBatchSolver(torch.from_numpy(Xn), opts).run(seeds)
    assert g.W.shape == (3 * K, 300) and bool((g.W >= 0).all())
    np.testing.assert_allclose(g.err, c.err, rtol=2e-3)
    assert np.abs(g.n_iter - c.n_iter).max() <= 2, (g.n_iter, c.n_iter)


@pytest.mark.parametrize("beta", [1.0, 0.0])
@pytest.mark.parametrize("conv_mode", [1, 0])
def test_split_bf16_h_block_rule_matches_reference(beta, conv_mode):
    """Multi-step usage blocks with the on-device stopping rule (last-arriving workgroup):
    iterate, flags, step counts and the block-objective state == the fp64 reference."""
    g = torch.Generator().manual_seed(7)
    R, K, N, G = 4, 10, 1500, 260
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    act0 = torch.tensor([1, 1, 0, 1], dtype=torch.int32)
    tol = 0.05 if conv_mode == 1 else 0.02
    nsteps = 5 if conv_mode == 1 else 1
    ref_h, ref_act = HT.clone(), act0.clone()
    ref_it, ref_hs = torch.zeros(R, dtype=torch.int32), torch.zeros((R, 2), dtype=torch.float64)
    gh, gact = HT.float().to(dev), act0.to(dev)
    git, ghs = torch.zeros(R, dtype=torch.int32, device=dev), torch.zeros(
        (R, 2), dtype=torch.float64, device=dev)
    Xg, Wg = X.float().to(dev), W.float().to(dev)
    pan = ops.beta_panels(Wg, beta)
    for blk in range(4):
        kw = dict(gamma=1.0 if beta else 0.5, tol=tol, conv_mode=conv_mode,
                  loss_entry=blk == 0)
        reference.beta_h_block(X, ref_h, W, beta, 1e-10, nsteps, 0.01, 0.0, act=ref_act,
                               iters=ref_it, hstate=ref_hs, **kw)
        ops.beta_h_block(Xg, gh, Wg, beta, 1e-10, nsteps, 0.01, 0.0, act=gact, iters=git,
                         hstate=ghs, panels=pan, **kw)
    # KL: fp16 numerator plane (see test_split_bf16_beta_kernels_match_fp64), 20 steps
    torch.testing.assert_close(gh.cpu().double(), ref_h, rtol=1e-3 if beta == 1.0 else 2e-4,
                               atol=1e-5)
    assert gact.cpu().tolist() == ref_act.tolist()
    assert git.cpu().tolist() == ref_it.tolist()
    if conv_mode == 1:
        torch.testing.assert_close(ghs.cpu(), ref_hs, rtol=1e-4, atol=1e-6)
    assert torch.equal(gh[2].cpu(), HT[2].float())           # inactive replicate untouched


@pytest.mark.parametrize("d", [7, 20, 50])
def test_kmeanspp_fused_step_matches_reference(d):
    """Fused k-means++ candidate scoring / closest update (kmeans.hip kmeanspp_kernel) vs
    the float64 torch reference; ragged n (not a multiple of the 256-point blocks)."""
    rs = np.random.default_rng(d)
    n, n_init, trials = 5000 + 37, 10, 6
    X = torch.from_numpy(rs.normal(size=(n, d)))
    C = torch.from_numpy(rs.normal(size=(n_init * trials, d)))
    closest = torch.from_numpy(rs.random((n, n_init)) * d)
    ref = ops.kmeanspp_step(X, C, closest.clone(), trials)
    got = ops.kmeanspp_step(X.cuda(), C.cuda(), closest.cuda().contiguous(), trials)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-11, atol=1e-9)
    ch = C[::trials].contiguous()
    cr, cg = closest.clone(), closest.cuda().contiguous()
    ops.kmeanspp_step(X, ch, cr, 1, update=True)
    ops.kmeanspp_step(X.cuda(), ch.cuda(), cg, 1, update=True)
    torch.testing.assert_close(cg.cpu(), cr, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n", [1000, 300000 + 37])
def test_kmeanspp_sample_matches_cumsum_searchsorted(n):
    """Device k-means++ draw (kmeans.hip ppsum/ppsample) == torch cumsum + searchsorted
    (side left, clamped), including u = 0 and u = 1 and zero-potential stretches; a
    zero-potential point is never drawn."""
    rs = np.random.default_rng(n)
    n_init, trials = 10, 6
    closest = torch.from_numpy(rs.random((n, n_init)) ** 3)
    closest[: n // 3, 2] = 0.0                   # a restart with a zero-potential prefix
    u = torch.from_numpy(rs.random((n_init, trials)))
    u[0, 0], u[1, 1], u[2, 0] = 0.0, 1.0, 1e-300
    cum = torch.cumsum(closest.t().contiguous(), 1)
    ref = torch.searchsorted(cum, u * cum[:, -1:]).clamp(max=n - 1)
    got = ops.kmeanspp_sample(closest.cuda().contiguous(), u.cuda()).cpu()
    # a draw may land one point over where the two summation orders round the running
    # sum differently right at the target; away from such ties the draws are identical
    diff = (got - ref).abs()
    assert int((diff > 0).sum()) <= 1 and int(diff.max()) <= 1
    assert got[0, 0] == 0 and got[2, 0] == n // 3
    # zeroed tails and u at (or a hair below) 1: the draw is the LAST point of positive
    # potential, never a zero-potential one past it (existing centres, padding)
    tail = closest.clone()
    last = (3 * n) // 5
    tail[last + 1:, :] = 0.0
    ut = torch.full((n_init, trials), 1.0 - 1e-16, dtype=torch.float64)
    ut[:, 0] = 1.0
    got_t = ops.kmeanspp_sample(tail.cuda().contiguous(), ut.cuda()).cpu()
    assert int(got_t.max()) <= last
    pos = tail.t() > 0
    assert bool(pos[torch.arange(n_init)[:, None], got_t].all())
    assert (got_t[:, 0] == last).all()


def test_device_kmeans_large_n_uses_fused_init():
    """Harmony-sized k-means (many points, few PCs) goes through the fused k-means++ path
    and still separates planted clusters."""
    from sklearn.metrics import adjusted_rand_score

    from cnmf_torch_amd.models.consensus import kmeans

    rs = np.random.default_rng(5)
    centers = rs.normal(size=(8, 20)) * 6
    truth = rs.integers(0, 8, 30000)
    X = torch.from_numpy(centers[truth] + rs.normal(size=(30000, 20))).cuda()
    assert ops.kmeanspp_fused_ok(X, 10 * (2 + int(np.log(8))))
    got = kmeans(X, 8, n_init=10, random_state=0, max_iter=25, backend="device",
                 device_restart_factor=1)
    assert adjusted_rand_score(truth, got) > 0.99


def test_pairwise_dist_and_knn_density():
    """f64 MFMA distance tiles + radix-select neighbour sums vs sklearn/numpy."""
    from sklearn.metrics import euclidean_distances

    rs = np.random.default_rng(0)
    A = rs.random((333, 130))
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    A[7] = A[3]                                   # exact duplicate -> ties at distance 0
    dev = torch.device("cuda")
    D = ops.pairwise_dist(torch.from_numpy(A).to(dev)).cpu().numpy()
    ref = euclidean_distances(A)
    np.testing.assert_allclose(D, ref, rtol=1e-9, atol=1e-7)
    assert np.all(np.diag(D) == 0.0)
    B = rs.random((70, 130))
    D2 = ops.pairwise_dist(torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev),
                           squared=True).cpu().numpy()
    np.testing.assert_allclose(D2, euclidean_distances(A, B, squared=True), rtol=1e-9, atol=1e-9)
    for k in (1, 2, 31, 333):
        got = ops.knn_sum(torch.from_numpy(ref).to(dev), k).cpu().numpy()
        exp = np.sort(ref, axis=1)[:, :k].sum(1)
        np.testing.assert_allclose(got, exp, rtol=1e-12, atol=1e-12)


def test_seg_argmin_and_device_kmeans():
    from sklearn.metrics import adjusted_rand_score

    from cnmf_torch_amd.models.consensus import kmeans

    rs = np.random.default_rng(1)
    D = rs.random((500, 4 * 7))
    lab, mn = ops.seg_argmin(torch.from_numpy(D).cuda(), 7)
    V = D.reshape(500, 4, 7)
    np.testing.assert_array_equal(lab.cpu().numpy(), V.argmin(2))
    np.testing.assert_allclose(mn.cpu().numpy(), V.min(2))
    centers = rs.normal(size=(5, 40)) * 5
    truth = rs.integers(0, 5, 600)
    X = centers[truth] + rs.normal(size=(600, 40))
    got = kmeans(torch.from_numpy(X).cuda(), 5, backend="device")
    assert adjusted_rand_score(truth, got) > 0.99


@pytest.mark.parametrize("n,d,k,n_init", [(5000, 20, 30, 3), (2049, 50, 100, 2), (700, 7, 5, 4),
                                          (3000, 64, 40, 1)])
def test_kmeans_step_fused_matches_reference(n, d, k, n_init):
    """Fused Lloyd step (kmeans.hip) vs the fp64 torch oracle: labels, per-cluster sums,
    counts and distances; bitwise deterministic across launches."""
    rs = np.random.default_rng(n + d)
    X = torch.from_numpy(rs.normal(size=(n, d)))
    C = torch.from_numpy(rs.normal(size=(n_init, k, d)))
    assert ops.kmeans_fused_ok(X.cuda(), k)
    lab_r, sums_r, cnt_r, mind_r = ops.kmeans_step(X, C, want_dist=True)
    lab_g, sums_g, cnt_g, mind_g = ops.kmeans_step(X.cuda(), C.cuda(), want_dist=True)
    lab_g2, sums_g2, _, _ = ops.kmeans_step(X.cuda(), C.cuda())
    torch.cuda.synchronize()
    agree = (lab_g.cpu() == lab_r).double().mean().item()
    assert agree > 0.999, agree       # exact-vs-expanded distance may flip near-ties only
    # sums/counts from the GPU labels must equal the oracle accumulation of those labels
    Xd = X.double()
    for r in range(n_init):
        s = torch.zeros((k, d), dtype=torch.float64).index_add_(0, lab_g[r].cpu(), Xd)
        torch.testing.assert_close(sums_g[r].cpu(), s, rtol=1e-12, atol=1e-10)
        c = torch.bincount(lab_g[r].cpu(), minlength=k).double()
        torch.testing.assert_close(cnt_g[r].cpu(), c)
    torch.testing.assert_close(mind_g.cpu(), mind_r, rtol=1e-9, atol=1e-9)
    assert torch.equal(lab_g, lab_g2) and torch.equal(sums_g, sums_g2)
    # frozen restarts are skipped, live ones unchanged
    live = torch.zeros(n_init, dtype=torch.int32)
    live[0] = 1
    lab_l, sums_l, _, _ = ops.kmeans_step(X.cuda(), C.cuda(), live=live)
    assert torch.equal(lab_l[0], lab_g[0]) and torch.equal(sums_l[0], sums_g[0])


def test_harmony_native_matches_cpu():
    """Fused R-update kernels (harmony.hip) == the torch block loop, same block order."""
    import pandas as pd

    from cnmf_torch_amd import ops as _ops
    from cnmf_torch_amd.models.harmony import run_harmony

    rs = np.random.default_rng(0)
    n, d = 900, 12
    types = rs.integers(0, 3, n)
    batch = rs.integers(0, 3, n)
    donor = rs.integers(0, 2, n)
    Z = rs.normal(size=(3, d))[types] * 3 + rs.normal(size=(3, d))[batch] * 2 + 0.3 * rs.normal(
        size=(n, d))
    meta = pd.DataFrame({"batch": pd.Categorical(batch.astype(str)),
                         "donor": pd.Categorical(donor.astype(str))})
    for vars_use in ("batch", ["batch", "donor"]):
        cpu = run_harmony(Z, meta, vars_use, max_iter_harmony=4, random_state=0, device="cpu")
        gpu = run_harmony(Z, meta, vars_use, max_iter_harmony=4, random_state=0, device="cuda")
        assert _ops.harmony_native_ok(torch.zeros(1, device="cuda"), gpu.K, gpu.Phi.shape[0])
        np.testing.assert_allclose(gpu.R, cpu.R, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(gpu.Z_corr, cpu.Z_corr, rtol=1e-6, atol=1e-8)
        assert gpu.kmeans_rounds == cpu.kmeans_rounds


def test_harmony_fused_round_matches_float64_reference():
    """One Harmony k-means round on the fused kernels (harmony.hip) against float64 torch
    on the host, from identical state: the centroid kernel vs Z_cos R^T, a block R update
    whose assign forms the distances itself vs the same update from an explicit distance
    matrix, and the round objective (assign sums + K x B cross term) vs harmonypy's
    formula -- all to 1e-10."""
    import math

    g = torch.Generator().manual_seed(4)
    N, d, K, nb_var = 3000, 20, 30, 2
    B_per = [3, 2]
    B = sum(B_per)
    Z = torch.randn((d, N), generator=g, dtype=torch.float64)
    Zc = Z / torch.linalg.vector_norm(Z, dim=0)
    R = torch.rand((K, N), generator=g, dtype=torch.float64)
    R = R / R.sum(dim=0)
    labels = [torch.randint(0, b, (N,), generator=g) for b in B_per]
    Phi = torch.cat([torch.nn.functional.one_hot(l, b).t().double() for l, b in zip(labels, B_per)])
    bidx = torch.stack([labels[0], labels[1] + B_per[0]]).to(torch.int32)
    sigma = torch.full((K,), 0.1, dtype=torch.float64)
    theta = torch.ones(B, dtype=torch.float64)
    Pr_b = Phi.sum(dim=1) / N
    dev = torch.device("cuda")
    ws = {}
    # centroids
    Zt = Zc.t().contiguous()
    Y = ops.harmony_centroids(Zt.to(dev), R.t().contiguous().to(dev), ws).cpu()
    torch.testing.assert_close(Y, Zc @ R.t(), rtol=1e-10, atol=1e-12)
    Y = Y / torch.linalg.vector_norm(Y, dim=0)
    # one block update, fused distances vs explicit distances
    E = torch.outer(R.sum(dim=1), Pr_b)
    O = R @ Phi.t()
    cells = torch.randperm(N, generator=g)[:700].to(torch.int32)
    out = {}
    for fused in (True, False):
        Rt = R.t().contiguous().to(dev)
        Eg, Og = E.clone().to(dev), O.clone().to(dev)
        obj = torch.zeros(2, dtype=torch.float64, device=dev)
        w = {}
        if fused:
            ops.harmony_block_update(Rt, None, sigma.to(dev), cells.to(dev), bidx.to(dev), Eg, Og,
                                     Pr_b.to(dev), theta.to(dev), w, Y=Y.contiguous().to(dev),
                                     Zt=Zt.to(dev), obj=obj)
        else:
            distT = (2 * (1 - Zc.t() @ Y)).contiguous().to(dev)
            ops.harmony_block_update(Rt, distT, sigma.to(dev), cells.to(dev), bidx.to(dev), Eg,
                                     Og, Pr_b.to(dev), theta.to(dev), w)
        out[fused] = (Rt.cpu(), Eg.cpu(), Og.cpu(), obj.cpu())
    for a, b in zip(out[True][:3], out[False][:3]):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-13)
    # the block's objective terms and the round objective
    Rn = out[True][0].t()
    dist = 2 * (1 - Y.t() @ Zc)
    cl = cells.long()
    km = (Rn[:, cl] * dist[:, cl]).sum()
    ent = (sigma[:, None] * torch.where(Rn[:, cl] > 0, Rn[:, cl] * torch.log(Rn[:, cl]),
                                        torch.zeros(()))).sum()
    torch.testing.assert_close(out[True][3], torch.stack([km, ent]), rtol=1e-10, atol=1e-12)
    En, On = out[True][1], out[True][2]
    res = torch.zeros(1, dtype=torch.float64, device=dev)
    obj = out[True][3].to(dev)
    ops.harmony_objective(On.to(dev), En.to(dev), sigma.to(dev), theta.to(dev), obj, res)
    cross = (sigma[:, None] * theta[None, :] * On * torch.log((On + 1) / (En + 1))).sum()
    torch.testing.assert_close(res.cpu()[0], km + ent + cross, rtol=1e-10, atol=1e-12)
    assert float(obj.abs().sum()) == 0.0          # the accumulators are reset
    assert math.isfinite(float(res.cpu()[0]))


@pytest.mark.parametrize("algo,K", [("mu", 3), ("mu", 10), ("mu", 13), ("hals", 10), ("hals", 16),
                                    ("mu", 20), ("hals", 24)])
@pytest.mark.parametrize("conv_mode", [0, 1])
def test_solve_register_resident_variant(algo, K, conv_mode):
    """variant='reg' (x, numer in VGPRs across iterations) == streaming == fp64 reference."""
    R, n = 4, 1000
    x0, numer, gram = _problem(R, K, n, seed=K + 7)
    dev = torch.device("cuda")
    outs = {}
    for variant in ("stream", "reg"):
        for max_iter, tol in ((6, -1.0), (300, 1e-4)):
            xg = x0.clone().to(dev)
            lin = torch.zeros(R, device=dev)
            quad = torch.zeros(R, device=dev)
            it = torch.zeros(R, dtype=torch.int32, device=dev)
            ops.solve(algo, xg, numer.to(dev), gram.to(dev), max_iter=max_iter, tol=tol,
                      lin_out=lin, quad_out=quad, iters_out=it, conv_mode=conv_mode,
                      check_every=5, variant=variant, coop=1)
            outs[(variant, tol)] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu())
    xr = x0.clone().double()
    reference.solve(ops.ALGOS[algo], xr, numer.double(), gram.double(), None, 6, -1.0,
                    0.0, 0.0, 0.0, 1e-16, None, None, None, 1, conv_mode, 5)
    torch.testing.assert_close(outs[("reg", -1.0)][0].double(), xr, rtol=2e-4, atol=1e-4)
    assert torch.equal(outs[("reg", -1.0)][0], outs[("stream", -1.0)][0])
    a, b = outs[("reg", 1e-4)], outs[("stream", 1e-4)]
    assert (a[3] - b[3]).abs().max() <= 5
    assert ((a[0] - b[0]).norm() / b[0].norm()) < 2e-3
    torch.testing.assert_close(a[1], b[1], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(a[2], b[2], rtol=1e-3, atol=1e-3)
    # coop split into resident slices
    xg = x0.clone().to(dev)
    ops.solve(algo, xg, numer.to(dev), gram.to(dev), max_iter=6, tol=-1.0, conv_mode=conv_mode,
              check_every=5, variant="reg", coop=3)
    assert torch.equal(xg.cpu(), outs[("reg", -1.0)][0])


@pytest.mark.parametrize("algo", ["mu", "hals"])
@pytest.mark.parametrize("K,n", [(3, 3900), (8, 4000), (10, 2600), (11, 3000), (12, 2048)])
def test_solve_resident_multi_column(algo, K, n):
    """Resident variant with U = ceil(n / 1024) columns per thread (numerator staged in
    LDS) == streaming variant bit for bit on fixed steps, == fp64 reference; with the
    loss stopping rule the two agree to fp32 summation order."""
    R = 3
    x0, numer, gram = _problem(R, K, n, seed=K + 101)
    dev = torch.device("cuda")
    outs = {}
    for variant in ("stream", "reg"):
        xg = x0.clone().to(dev)
        ops.solve(algo, xg, numer.to(dev), gram.to(dev), max_iter=7, tol=-1.0, conv_mode=0,
                  variant=variant, coop=1)
        outs[variant] = xg.cpu()
    assert torch.equal(outs["reg"], outs["stream"])
    xr = x0.clone().double()
    reference.solve(ops.ALGOS[algo], xr, numer.double(), gram.double(), None, 7, -1.0,
                    0.0, 0.0, 0.0, 1e-16, None, None, None, 1, 0, 5)
    torch.testing.assert_close(outs["reg"].double(), xr, rtol=2e-4, atol=1e-4)
    res = {}
    for variant in ("stream", "reg"):
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        ops.solve(algo, xg, numer.to(dev), gram.to(dev), max_iter=200, tol=1e-4, conv_mode=1,
                  check_every=5, lin_out=lin, quad_out=quad, variant=variant, coop=1)
        res[variant] = (xg.cpu(), lin.cpu(), quad.cpu())
    a, b = res["reg"], res["stream"]
    assert ((a[0] - b[0]).norm() / b[0].norm()) < 2e-3
    torch.testing.assert_close(a[1], b[1], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(a[2], b[2], rtol=1e-3, atol=1e-3)


def test_solve_resident_rejects_oversized_slice():
    """A slice wider than res_max_cols(K) * 1024 columns cannot run resident."""
    K, n = 12, 4000                                   # U would be 4 > res_max_cols(12) = 2
    x0, numer, gram = _problem(1, K, n, seed=1)
    with pytest.raises(RuntimeError):
        ops.solve("mu", x0.cuda(), numer.cuda(), gram.cuda(), max_iter=2, variant="reg",
                  coop=1)
    assert ops._hip.solve_reg_max_cols(12) == 2048
    assert ops._hip.solve_reg_max_cols(10) == 3072


def test_online_pass_graph_replay_matches_eager(monkeypatch):
    """Passes replayed from a captured HIP graph == eagerly launched passes, bit for bit."""
    from cnmf_torch_amd.models.nmf import run_nmf_batch

    rs = np.random.default_rng(3)
    N, G, K = 3000, 500, 7
    X = (rs.gamma(1, 1, (N, K)) @ rs.gamma(0.5, 1, (K, G)) + 0.1 * rs.random((N, G))).astype(
        np.float32)
    kw = dict(online_chunk_size=1000, online_max_pass=8, tol=1e-6)
    seeds = list(range(40, 52))
    monkeypatch.setenv("CNMF_GRAPHS", "1")
    g = run_nmf_batch(X, K, seeds, device="cuda", **kw)
    monkeypatch.setenv("CNMF_GRAPHS", "0")
    e = run_nmf_batch(X, K, seeds, device="cuda", **kw)
    np.testing.assert_array_equal(g.W.cpu().numpy(), e.W.cpu().numpy())
    np.testing.assert_array_equal(g.err, e.err)
    np.testing.assert_array_equal(g.n_iter, e.n_iter)
    assert (g.n_iter >= 1).all() and (g.n_iter <= 8).all()   # passes counted on device


def test_run_concurrent_streams_match_serial_groups():
    """Two replicate groups on two HIP streams (shared coop budget) == each group alone."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions

    rs = np.random.default_rng(5)
    N, G, K = 4000, 600, 9
    X = torch.from_numpy((rs.gamma(1, 1, (N, K)) @ rs.gamma(0.5, 1, (K, G)) +
                          0.1 * rs.random((N, G))).astype(np.float32)).cuda()
    solver = NMFBatchSolver(X, NMFOptions(n_components=K, online_chunk_size=1500,
                                          online_max_pass=6))
    seeds = list(range(100, 132))
    both = solver.run_concurrent(seeds, n_streams=2)
    with ops.coop_share(2):      # same cooperative split as inside run_concurrent
        a = solver.run(seeds[:16])
        b = solver.run(seeds[16:])
    np.testing.assert_array_equal(both.W.cpu().numpy(),
                                  torch.cat([a.W, b.W]).cpu().numpy())
    np.testing.assert_array_equal(both.err, np.concatenate([a.err, b.err]))


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                  HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 10_000), R=st.integers(1, 6), K=st.integers(1, 32),
       n=st.integers(1, 5000), algo=st.sampled_from(["mu", "hals"]),
       pad=st.integers(0, 7), coop=st.sampled_from(["auto", 1, 3]),
       variant=st.sampled_from(["auto", "stream"]))
def test_solve_random_shapes_match_reference(seed, R, K, n, algo, pad, coop, variant):
    """Random (R, K, n), padded leading dimensions (strided views), both variants and
    cooperative splits: fixed-step results == fp64 reference."""
    g = torch.Generator().manual_seed(seed)
    W = torch.rand((R, K, 2 * K + 3), generator=g, dtype=torch.float64) + 0.05
    gram = torch.bmm(W, W.transpose(1, 2))
    numer = torch.rand((R, K, n), generator=g, dtype=torch.float64) * K
    x0 = torch.rand((R, K, n), generator=g, dtype=torch.float64) + 0.1
    dev = torch.device("cuda")
    xs = torch.zeros((R, K, n + pad), device=dev)
    xs[:, :, :n] = x0.float().to(dev)
    xv = xs[:, :, :n]                                     # ldx = n + pad
    ops.solve(algo, xv, numer.float().to(dev), gram.float().to(dev), max_iter=3, tol=-1.0,
              coop=coop, variant=variant)
    xr = x0.clone()
    reference.solve(ops.ALGOS[algo], xr, numer, gram, None, 3, -1.0, 0.0, 0.0, 0.0, 1e-16,
                    None, None, None, 1, 0, 10)
    torch.testing.assert_close(xv.cpu().double(), xr, rtol=5e-4, atol=5e-4)
    assert torch.all(xs[:, :, n:] == 0)                   # padding untouched
    ops.coop_check(dev)


@pytest.mark.parametrize("K", [1, 5, 10, 16, 17, 32])
def test_gram_column_split_matches_single_workgroup(K):
    """Few replicates (column-split Gram + ordered reduce) == many-replicate path (one
    workgroup per replicate) on the same blocks, to fp32 summation order."""
    g = torch.Generator().manual_seed(K + 1)
    H = torch.rand((80, K, 5000), generator=g).cuda()
    full = ops.gram(H)                      # R = 80: one workgroup per replicate
    few = ops.gram(H[:8])                   # R = 8: S column slices per replicate
    torch.testing.assert_close(few, full[:8], rtol=2e-6, atol=1e-3)
    assert torch.equal(few, ops.gram(H[:8]))          # deterministic


@pytest.mark.parametrize("K", [1, 5, 10, 16, 17, 20, 32])
def test_gram_kernel_matches_bmm(K):
    """MFMA batched Gram (gram.hip): strided / offset views, ragged n, accumulate, active."""
    g = torch.Generator().manual_seed(K)
    R, N = 5, 1237
    H = torch.rand((R, K, N), generator=g, dtype=torch.float64)
    dev = torch.device("cuda")
    Hd = H.float().to(dev)
    for a, b in ((0, N), (3, 1001), (17, 18), (5, 5)):
        view = Hd[:, :, a:b]                                 # unaligned base, ragged width
        ref = torch.bmm(H[:, :, a:b], H[:, :, a:b].transpose(1, 2))
        got = ops.gram(view)
        torch.testing.assert_close(got.cpu().double(), ref, rtol=1e-5, atol=1e-4)
    out = torch.full((R, K, K), 2.0, device=dev)
    active = torch.tensor([1, 0, 1, 1, 0], dtype=torch.int32, device=dev)
    ops.gram(Hd, out=out, accumulate=True, active=active)
    ref = 2.0 + torch.bmm(H, H.transpose(1, 2))
    for r in range(R):
        if active[r]:
            torch.testing.assert_close(out[r].cpu().double(), ref[r], rtol=1e-5, atol=1e-3)
        else:
            assert torch.all(out[r] == 2.0)


@pytest.mark.parametrize("beta", [1.0, 0.0, 1.5])
def test_beta_w_update_matches_reference(beta):
    """Anchored online spectra step (beta_w_update_kernel) vs the float64 reference,
    including the on-device relative-change stop and inactive replicates."""
    g = torch.Generator().manual_seed(5)
    R, K, N, G = 4, 7, 500, 333
    gamma = 0.5 if beta < 1 else 1.0
    kl = beta == 1.0
    X = torch.rand((N, G), generator=g, dtype=torch.float64) + 0.05
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.1
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.1
    An = torch.rand((R, K, G), generator=g, dtype=torch.float64)
    Ad = torch.rand((R, K) if kl else (R, K, G), generator=g, dtype=torch.float64) + 0.5
    dev = torch.device("cuda")
    act0 = torch.tensor([1, 0, 1, 1], dtype=torch.int32)
    hsum = HT.sum(dim=2) if kl else None
    # CPU reference (float64)
    Wr, anr = W.clone(), torch.zeros_like(W)
    dnr = None if kl else torch.zeros_like(W)
    ar, itr = act0.clone(), torch.zeros(R, dtype=torch.int32)
    # GPU
    Wg = W.float().to(dev)
    ang = torch.zeros((R, K, G), device=dev)
    dng = None if kl else torch.zeros((R, K, G), device=dev)
    ag, itg = act0.to(dev), torch.zeros(R, dtype=torch.int32, device=dev)
    for _ in range(3):
        nr, dr, _ = reference.beta_contract(1, X, HT, Wr, beta, 1e-10, True, False)
        reference.beta_w_update(Wr, nr.unsqueeze(0), None if kl else dr.unsqueeze(0), hsum, An,
                                Ad, anr, dnr, beta, gamma, 0.01, 0.02, 1e-10, 1e-3, ar, itr)
        ng, dg, _ = ops.beta_contract("w", X.float().to(dev), HT.float().to(dev), Wg, beta,
                                      1e-10, active=ag, reduce=False)
        ops.beta_w_update(Wg, ng, dg, hsum.float().to(dev) if kl else None,
                          An.float().to(dev), Ad.float().to(dev), ang, dng, beta, gamma, 0.01,
                          0.02, 1e-10, 1e-3, ag, itg)
    torch.cuda.synchronize()
    live = [0, 2, 3]
    torch.testing.assert_close(Wg.cpu().double()[live], Wr[live], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ang.cpu().double()[live], anr[live], rtol=1e-4, atol=1e-4)
    assert torch.equal(Wg[1].cpu(), W[1].float())            # inactive replicate untouched
    assert itg.cpu().tolist() == itr.tolist()
    assert ag.cpu().tolist() == ar.tolist()


def test_beta_update_h_loss_rule_matches_reference():
    """conv_mode 1 (block beta-divergence every check_every steps) on device == reference."""
    g = torch.Generator().manual_seed(6)
    R, K, N, G = 5, 6, 900, 210
    X = torch.rand((N, G), generator=g, dtype=torch.float64) + 0.02
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    hr, ar = HT.clone(), torch.ones(R, dtype=torch.int32)
    itr, hsr = torch.zeros(R, dtype=torch.int32), torch.zeros((R, 2), dtype=torch.float64)
    hg, ag = HT.float().to(dev), torch.ones(R, dtype=torch.int32, device=dev)
    itg = torch.zeros(R, dtype=torch.int32, device=dev)
    hsg = torch.zeros((R, 2), dtype=torch.float64, device=dev)
    Xg, Wg = X.float().to(dev), W.float().to(dev)
    for _ in range(40):
        reference.beta_update_h(X, hr, W, 1.0, 1e-10, act=ar, tol=0.02, iters=itr, conv_mode=1,
                                check_every=4, hstate=hsr)
        ops.beta_update_h(Xg, hg, Wg, 1.0, 1e-10, act=ag, tol=0.02, iters=itg, conv_mode=1,
                          check_every=4, hstate=hsg)
    torch.cuda.synchronize()
    assert itg.cpu().tolist() == itr.tolist(), (itg, itr)
    assert ag.cpu().tolist() == ar.tolist()
    torch.testing.assert_close(hsg.cpu()[:, 0], hsr[:, 0], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(hg.cpu().double(), hr, rtol=2e-4, atol=1e-5)


@pytest.mark.parametrize("beta_loss", ["kullback-leibler", "itakura-saito"])
def test_online_beta_gpu_converges_like_cpu(beta_loss):
    """Online beta-MU on the GPU converges (flags, passes) and lands within 1 % of batch,
    with passes / inner iteration counts close to the CPU run of the same algorithm."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 400, n_programs=6, seed=0))
    kw = dict(beta_loss=beta_loss, online_chunk_size=1000, online_chunk_max_iter=1000,
              batch_max_iter=2000)
    seeds = [1, 2, 3]
    on_g = NMFBatchSolver(X.cuda(), NMFOptions(n_components=6, mode="online", **kw)).run(seeds)
    on_c = NMFBatchSolver(X, NMFOptions(n_components=6, mode="online", **kw)).run(seeds)
    ba_g = NMFBatchSolver(X.cuda(), NMFOptions(n_components=6, mode="batch", **kw)).run(seeds)
    assert on_g.converged.all() and (on_g.n_iter < 20).all(), on_g.n_iter
    assert (np.abs(on_g.err - ba_g.err) / ba_g.err < 0.01).all(), (on_g.err, ba_g.err)
    np.testing.assert_allclose(on_g.err, on_c.err, rtol=5e-3)
    assert np.abs(on_g.n_iter - on_c.n_iter).max() <= 3, (on_g.n_iter, on_c.n_iter)


def test_kl_fp16_numerator_overflow_is_redone_with_a_shift(kl_fp16):
    """x / p far beyond the fp16 range (65504) in a few (cell, gene) entries: the KL kernels
    redo such a step with the affected columns' Q shifted by 2^-12 (beta_planes.hip), so
    usages, spectra partials and the loss stay finite and match the float64 reference."""
    g = torch.Generator().manual_seed(3)
    R, K, N, G = 2, 10, 700, 300
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    X[X < 0.3] = 0.0
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    X[5, 7] = 3e6                     # p ~ 1: x / p ~ 3e6 and 2e9 (two shifts)
    X[400, 250] = 2e9
    X[699, 0] = 1e5
    dev = torch.device("cuda")
    eps = 1e-10
    Xg, Hg, Wg = X.float().to(dev), HT.float().to(dev), W.float().to(dev)
    h1 = Hg.clone()
    ops.beta_h_block(Xg, h1, Wg, 1.0, eps, 3)
    h2 = HT.clone()
    reference.beta_h_block(X, h2, W, 1.0, eps, 3)
    assert torch.isfinite(h1).all()
    # the shifted columns' sums are dominated by one huge term, so their fp16 rounding
    # (2^-11) does not average out: 5e-3 after three steps
    torch.testing.assert_close(h1.cpu().double(), h2, rtol=5e-3, atol=1e-6)
    rn, _, _ = reference.beta_contract(1, X, HT, W, 1.0, eps, True, False)
    num, _ = ops.beta_w_partials(Xg, Xg.t().contiguous(), Hg, Wg, 1.0, eps, splits=2)
    assert torch.isfinite(num).all()
    torch.testing.assert_close(num.sum(0).cpu().double(), rn, rtol=1e-3, atol=1e-5)


def test_kl_fp16_count_operands_match_fp64(monkeypatch):
    """KL kernels reading X as fp16 counts (X = C u_g; P panel of W / u, loss weights u,
    spectra side's W scaled by 1 / u) vs the float64 reference on the fp32 X: the
    fp16-numerator kernels on both sides, and the default (fp32-accurate) KL spectra side,
    the one the engine feeds counts, at its 5e-5."""
    monkeypatch.setenv("CNMF_KL_FP16", "1")
    ops.refresh_env()
    g = torch.Generator().manual_seed(5)
    R, K, N, G = 3, 10, 777, 300
    C = torch.poisson(torch.rand((N, G), generator=g, dtype=torch.float64) * 3)
    u = torch.rand(G, generator=g, dtype=torch.float64) * 2 + 0.1
    X = C * u
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    eps = 1e-10
    Xg, Hg, Wg = X.float().to(dev), HT.float().to(dev), W.float().to(dev)
    ug = u.float().to(dev)
    xh = C.to(torch.float16).to(dev)
    pan = ops.beta_panels(Wg, 1.0, row_scale=(1.0 / ug).contiguous())
    h1 = Hg.clone()
    act = torch.ones(R, dtype=torch.int32, device=dev)
    hs = torch.zeros((R, 2), dtype=torch.float64, device=dev)
    ops.beta_h_block(Xg, h1, Wg, 1.0, eps, 4, act=act, tol=1e-12, hstate=hs, loss_entry=True,
                     panels=pan, xh=xh, unit=ug)
    h2 = HT.clone()
    act_r = torch.ones(R, dtype=torch.int32)
    hs_r = torch.zeros((R, 2), dtype=torch.float64)
    reference.beta_h_block(X, h2, W, 1.0, eps, 4, act=act_r, tol=1e-12, hstate=hs_r,
                           loss_entry=True)
    torch.testing.assert_close(h1.cpu().double(), h2, rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(hs.cpu()[:, 0], hs_r[:, 0], rtol=1e-4, atol=1e-3)
    rn, _, _ = reference.beta_contract(1, X, HT, W, 1.0, eps, True, False)
    num, _ = ops.beta_w_partials(Xg, None, Hg, Wg, 1.0, eps, splits=2,
                                 xth=xh.t().contiguous(), unit_inv=(1.0 / ug).contiguous())
    torch.testing.assert_close(num.sum(0).cpu().double(), rn, rtol=5e-4, atol=1e-5)
    with pytest.raises(ValueError):        # row-scaled panels without the counts
        ops.beta_h_block(Xg, Hg.clone(), Wg, 1.0, eps, 1, panels=pan)
    monkeypatch.delenv("CNMF_KL_FP16")
    ops.refresh_env()
    num, _ = ops.beta_w_partials(Xg, None, Hg, Wg, 1.0, eps, splits=2,
                                 xth=xh.t().contiguous(), unit_inv=(1.0 / ug).contiguous())
    torch.testing.assert_close(num.sum(0).cpu().double(), rn, rtol=5e-5, atol=1e-5)


@pytest.mark.parametrize("numer", ["default", "fp16"])
def test_online_kl_matches_fp32_torch_path(numer, monkeypatch):
    """Online KL through the split-bf16 kernels (default fp32-accurate numerator; opt-in
    fp16 one) vs the same solver on plain fp32 PyTorch ops (CNMF_FORCE_TORCH_OPS=1):
    final objectives within 1e-4 (fp16: 1e-3), passes within 1."""
    if numer == "fp16":
        monkeypatch.setenv("CNMF_KL_FP16", "1")
    ops.refresh_env()
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 400, n_programs=6, seed=0)).cuda()
    opts = NMFOptions(n_components=6, beta_loss="kullback-leibler", online_chunk_size=1000,
                      online_chunk_max_iter=1000)
    seeds = [1, 2, 3, 4]
    a = NMFBatchSolver(X, opts).run(seeds)
    old = os.environ.get("CNMF_FORCE_TORCH_OPS")
    os.environ["CNMF_FORCE_TORCH_OPS"] = "1"
    ops.refresh_env()
    try:
        b = NMFBatchSolver(X, opts).run(seeds)
    finally:
        if old is None:
            os.environ.pop("CNMF_FORCE_TORCH_OPS")
        else:
            os.environ["CNMF_FORCE_TORCH_OPS"] = old
        ops.refresh_env()
    assert a.converged.all() and b.converged.all()
    np.testing.assert_allclose(a.err, b.err, rtol=1e-3 if numer == "fp16" else 1e-4)
    assert np.abs(a.n_iter - b.n_iter).max() <= 1, (a.n_iter, b.n_iter)
    monkeypatch.delenv("CNMF_KL_FP16", raising=False)
    ops.refresh_env()


@pytest.mark.parametrize("K,G", [(3, 333), (10, 333), (17, 333), (32, 1200)])
def test_sparse_kl_kernels_match_fp64(K, G):
    """sparse_kl.hip (CSR X, fp32 gathers) vs the float64 dense reference: a 3-step usage
    block with the block-objective rule, the spectra numerators and the loss (W^T staged
    in LDS; K = 32, G = 1200 exceeds the LDS budget and gathers from L2)."""
    g = torch.Generator().manual_seed(K)
    R, N = 3, 901
    X = torch.rand((N, G), generator=g, dtype=torch.float64)
    X[X < 0.85] = 0.0                                   # ~15 % dense
    X[7] = 0.0                                          # an empty row
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) + 0.05
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64) + 0.05
    dev = torch.device("cuda")
    eps = 1e-10
    Xg, Hg, Wg = X.float().to(dev), HT.float().to(dev), W.float().to(dev)
    csr = ops.kl_csr(Xg)
    assert int(csr.rowptr[-1]) == int((X != 0).sum())
    # loss
    ref_loss = reference.beta_contract(0, X, HT, W, 1.0, eps, False, True)[2]
    torch.testing.assert_close(ops.kl_sparse_loss(csr, Hg, Wg, eps).cpu(), ref_loss, rtol=1e-5,
                               atol=1e-6)
    # spectra numerators over a row chunk
    a, b = 100, 700
    rn, _, _ = reference.beta_contract(1, X[a:b], HT[:, :, a:b], W, 1.0, eps, True, False)
    tiles = ops.kl_csr_tiles(Xg[a:b], K)
    num = ops.kl_sparse_w_num(tiles, Hg[:, :, a:b].contiguous(), Wg, eps)
    torch.testing.assert_close(num.sum(0).cpu().double(), rn, rtol=2e-5, atol=1e-6)
    # several LDS tiles (forced small) == one
    t2 = [(t0, ops.kl_csr(Xg[a + t0:a + min(b - a, t0 + 128)].t())) for t0 in range(0, b - a, 128)]
    num2 = ops.kl_sparse_w_num(t2, Hg[:, :, a:b].contiguous(), Wg, eps)
    torch.testing.assert_close(num2.sum(0), num.sum(0), rtol=1e-5, atol=1e-6)
    # usage block with the rule, on a row range of the CSR (rowptr slice)
    h1 = Hg[:, :, a:b].contiguous()
    h2 = HT[:, :, a:b].clone()
    act_g = torch.ones(R, dtype=torch.int32, device=dev)
    act_r = torch.ones(R, dtype=torch.int32)
    it_g = torch.zeros(R, dtype=torch.int32, device=dev)
    it_r = torch.zeros(R, dtype=torch.int32)
    hs_g = torch.zeros((R, 2), dtype=torch.float64, device=dev)
    hs_r = torch.zeros((R, 2), dtype=torch.float64)
    for blk in range(3):
        ops.kl_sparse_h_block(ops.kl_csr_rows(csr, a, b), h1, Wg, eps, 3, 0.01, 0.0, act=act_g,
                              tol=0.05, iters=it_g, hstate=hs_g, loss_entry=blk == 0)
        reference.beta_h_block(X[a:b], h2, W, 1.0, eps, 3, 0.01, 0.0, act=act_r, tol=0.05,
                               iters=it_r, hstate=hs_r, loss_entry=blk == 0)
    torch.testing.assert_close(h1.cpu().double(), h2, rtol=1e-4, atol=1e-6)
    assert act_g.cpu().tolist() == act_r.tolist()
    assert it_g.cpu().tolist() == it_r.tolist()
    torch.testing.assert_close(hs_g.cpu(), hs_r, rtol=1e-5, atol=1e-6)


def test_online_kl_sparse_path_matches_dense():
    """Online KL on a ~15 %-dense matrix: the CSR kernels (CNMF_KL_SPARSE=1) and the dense
    split-precision kernels (=0) give the same factorisation."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = normalized_counts_matrix(3000, 400, n_programs=6, seed=0)
    X[X < np.quantile(X, 0.85)] = 0.0
    Xg = torch.from_numpy(X).cuda()
    opts = NMFOptions(n_components=6, beta_loss="kullback-leibler", online_chunk_size=1000,
                      online_chunk_max_iter=1000)
    res = {}
    old = os.environ.get("CNMF_KL_SPARSE")
    try:
        for flag in ("1", "0"):
            os.environ["CNMF_KL_SPARSE"] = flag
            s = NMFBatchSolver(Xg, opts)
            res[flag] = s.run([1, 2, 3])
            assert (s._kl_sparse() is not None) == (flag == "1")
    finally:
        if old is None:
            os.environ.pop("CNMF_KL_SPARSE", None)
        else:
            os.environ["CNMF_KL_SPARSE"] = old
    a, b = res["1"], res["0"]
    assert a.converged.all()
    np.testing.assert_allclose(a.err, b.err, rtol=2e-3)
    assert np.abs(a.n_iter - b.n_iter).max() <= 1, (a.n_iter, b.n_iter)


@pytest.mark.parametrize("density,sparse", [(0.08, True), (0.17, True), (0.21, False),
                                            (0.47, False)])
def test_kl_sparse_routing_follows_measured_crossover(monkeypatch, density, sparse):
    """Without CNMF_KL_SPARSE, KL takes the CSR kernels up to kl_sparse_density (0.18,
    the measured crossover: profiles/r4h_kl_*) and the dense kernels above it."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    monkeypatch.delenv("CNMF_KL_SPARSE", raising=False)
    X = normalized_counts_matrix(2000, 300, n_programs=5, seed=1)
    X[X < np.quantile(X, 1.0 - density)] = 0.0
    s = NMFBatchSolver(torch.from_numpy(X).cuda(),
                       NMFOptions(n_components=5, beta_loss="kullback-leibler"))
    assert NMFOptions(n_components=5).kl_sparse_density == 0.18
    assert (s._kl_sparse() is not None) == sparse


def test_online_kl_without_xt_copy_matches():
    """When X^T does not fit beside X the spectra side falls back to the fp32 kernel that
    reads X in place (beta_mu.hip): same factorisation as the split-bf16 X^T path."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 400, n_programs=6, seed=0)).cuda()
    opts = NMFOptions(n_components=6, beta_loss="kullback-leibler", online_chunk_size=1000,
                      online_chunk_max_iter=1000)
    a = NMFBatchSolver(X, opts).run([1, 2])
    s = NMFBatchSolver(X, opts)
    s._XT = False                       # as if the second copy of X had not fit
    b = s.run([1, 2])
    assert s._xt() is None
    np.testing.assert_allclose(a.err, b.err, rtol=2e-3)
    assert np.abs(a.n_iter - b.n_iter).max() <= 2, (a.n_iter, b.n_iter)


def test_refit_raises_when_a_cooperative_solve_timed_out():
    """A raised cooperative-timeout flag (workgroups not co-resident) must surface as an
    error from the usage refit, and the kernels must stop waiting on it."""
    from cnmf_torch_amd.models.refit import fit_H_online

    rs = np.random.default_rng(1)
    X = rs.random((3000, 200)).astype(np.float32)
    W = rs.random((5, 200)).astype(np.float32)
    H = fit_H_online(X, W, chunk_size=3000, device="cuda")     # one chunk -> coop split
    assert np.isfinite(H).all()
    dev = torch.device("cuda", torch.cuda.current_device())
    ws = ops._COOP_WS.get((str(dev), torch.cuda.current_stream().cuda_stream))
    assert ws is not None, "the refit did not take the cooperative path"
    ws["flag"].fill_(1)
    with pytest.raises(RuntimeError, match="cooperative solve failed"):
        fit_H_online(X, W, chunk_size=3000, device="cuda")
    ops.coop_check(torch.device("cuda"))    # flag consumed by the raise: clean again
    assert int(ws["flag"].item()) == 0


@pytest.mark.parametrize("mode", ["online", "batch"])
def test_mixed_k_ragged_batch_gpu_matches_single_k(mode):
    """The K x n_iter grid as ONE ragged batch on the GPU == per-K batches."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions

    rs = np.random.default_rng(3)
    N, G = 2000, 300
    X = torch.from_numpy((rs.gamma(1, 1, (N, 8)) @ rs.gamma(0.5, 1, (8, G))
                          + 0.1 * rs.random((N, G))).astype(np.float32)).cuda()
    kw = dict(mode=mode, online_chunk_size=900, online_max_pass=8, batch_max_iter=60)
    ks = [5, 7, 5, 13, 7, 13, 5, 7, 24, 5]
    seeds = list(range(31, 41))
    mixed = NMFBatchSolver(X, NMFOptions(n_components=5, **kw)).run(seeds, ks=ks)
    for K in sorted(set(ks)):
        idx = [i for i, k in enumerate(ks) if k == K]
        ref = NMFBatchSolver(X, NMFOptions(n_components=K, **kw)).run([seeds[i] for i in idx])
        for j, i in enumerate(idx):
            assert abs(int(mixed.n_iter[i]) - int(ref.n_iter[j])) <= 1
            np.testing.assert_allclose(mixed.err[i], ref.err[j], rtol=2e-3)
            a, b = mixed.spectra(i).cpu().numpy(), ref.spectra(j).cpu().numpy()
            cos = (a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))
            assert cos.min() > 0.98, cos


@pytest.mark.parametrize("rows,cols", [(37, 50), (300, 2000), (1, 7)])
def test_split_planes_bitwise_matches_reference(rows, cols):
    g = torch.Generator().manual_seed(rows)
    S = (torch.rand((rows, cols), generator=g) * 50 - 5) ** 3
    mul = torch.rand(cols, generator=g) + 0.5
    ld = -(-cols // 64) * 64
    out = torch.zeros((3, rows, ld), dtype=torch.int16, device="cuda")
    ops.split_planes(S.cuda(), out, col_mul=mul.cuda())
    ref = reference.split_planes(S * mul, 3, ld)
    assert torch.equal(out.cpu(), ref)
    # exact: the planes sum back to the scaled fp32 input
    back = reference.planes_to_f64(out.cpu()).sum(0)[:, :cols]
    assert torch.equal(back.float(), S * mul)


@pytest.mark.parametrize("pb", [1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(1000, 5000, 2000), (83, 130, 96), (8100, 700, 320)])
def test_gemm_planes_matches_fp64(pb, M, N, K):
    """Split-precision MFMA GEMM == the fp64 product to fp32-GEMM accuracy, including
    ragged edges, a B row offset, accumulation and a per-column output scale."""
    g = torch.Generator().manual_seed(M + N + pb)
    bk = ops.planes_bk(pb)
    Kd = -(-K // bk) * bk
    A = torch.rand((M, K), generator=g)
    if pb < 3:   # integer "counts" held exactly in pb planes
        B = torch.randint(0, 200 if pb == 1 else 3000, (N + 40, K), generator=g).float()
    else:
        B = torch.rand((N + 40, K), generator=g)
    scale = torch.rand(N, generator=g) + 0.5
    Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device="cuda")
    Bp = torch.zeros((pb, N + 40, Kd), dtype=torch.int16, device="cuda")
    ops.split_planes(A.cuda(), Ap)
    ops.split_planes(B.cuda(), Bp)
    if pb < 3:
        assert torch.equal(reference.planes_to_f64(Bp.cpu()).sum(0)[:, :K], B.double())
    C0 = torch.rand((M, N), generator=g)
    C = C0.clone().cuda()
    ops.gemm_planes(C, Ap, Bp[:, 40:], M, N, Kd, accumulate=True, col_scale=scale.cuda())
    ref = C0.double() + (A.double() @ B[40:].double().t()) * scale.double()
    err = (C.cpu().double() - ref).abs().max() / ref.abs().max()
    # an fp32 GEMM over K terms: ~K * 2^-24 worst case, far less in practice (hipBLASLt's
    # fp32 GEMM: 3.5e-6 at K = 2000, profiles/r2_gemm_planes_sweep.log; unsplit k here)
    tol = 1e-6 * max(1.0, K / 256)
    assert err < tol, float(err)
    C2 = torch.empty((M, N), device="cuda")
    ops.gemm_planes(C2, Ap, Bp[:, 40:], M, N, Kd)
    ref2 = A.double() @ B[40:].double().t()
    assert float((C2.cpu().double() - ref2).abs().max() / ref2.abs().max()) < tol


def test_count_units_detects_scaled_counts():
    from cnmf_torch_amd.models.nmf import _XPlanes, _count_units

    rs = np.random.default_rng(0)
    C = rs.poisson(rs.gamma(0.3, 3, (1, 400)), (3000, 400)).astype(np.float64)
    C[:, 5] = 0
    C[:, 7] = 2 * rs.integers(1, 5, 3000)          # smallest count 2
    std = C.std(0, ddof=1)
    std[std == 0] = 1
    X = torch.from_numpy((C / std).astype(np.float32)).cuda()
    u = _count_units(X)
    assert u is not None
    back = torch.round(X / u) * u
    assert float(((back - X).abs() / X.abs().clamp(min=1e-30)).max()) < 3e-7
    xp = _XPlanes(X)
    assert xp.pb == (1 if C.max() <= 256 else 2)
    assert _count_units(X + 0.01 * torch.rand_like(X)) is None


def test_split_gemm_solver_matches_fp32_library_gemm(monkeypatch):
    """The NMF solve with the split-precision MFMA GEMMs == the same solve on the fp32
    library GEMMs (CNMF_GEMM=torch) to fp32 reassociation noise."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 500, n_programs=6, seed=1)).cuda()
    kw = dict(online_chunk_size=1000, online_max_pass=10)
    seeds = list(range(1, 9))
    ks = [5, 6, 7, 6, 5, 7, 9, 9]
    planes = NMFBatchSolver(X, NMFOptions(n_components=5, **kw))
    a = planes.run(seeds, ks=ks)
    assert planes._planes() is not None and planes._planes().pb in (1, 2)
    monkeypatch.setenv("CNMF_GEMM", "torch")
    lib = NMFBatchSolver(X, NMFOptions(n_components=5, **kw))
    b = lib.run(seeds, ks=ks)
    assert lib._planes() is None
    np.testing.assert_allclose(a.err, b.err, rtol=1e-4)
    assert np.abs(a.n_iter - b.n_iter).max() <= 1


def test_coop_solve_with_a_concurrent_kernel_stream():
    """Cooperative (spin-waiting) solves while another stream keeps the chip busy (the
    situation of an RCCL kernel resident beside the solver under DP): results equal the
    isolated solve and no cooperative wait gives up."""
    x0, numer, gram = _problem(6, 10, 20000, seed=11)
    ref_x = x0.clone().cuda()
    ops.solve("mu", ref_x, numer.cuda(), gram.cuda(), max_iter=200, tol=1e-4, conv_mode=1)
    side = torch.cuda.Stream()
    big = torch.rand((4096, 4096), device="cuda")
    x = x0.clone().cuda()
    nu, gr = numer.cuda(), gram.cuda()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(20):
            big = torch.tanh(big @ big * 1e-3)
    for _ in range(3):
        x.copy_(x0.cuda())
        ops.solve("mu", x, nu, gr, max_iter=200, tol=1e-4, conv_mode=1)
    torch.cuda.synchronize()
    ops.coop_check(torch.device("cuda"))
    np.testing.assert_allclose(x.cpu().numpy(), ref_x.cpu().numpy(), rtol=1e-5, atol=1e-7)


def test_colstats_and_count_unit_check_match_reference():
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3001, 517, n_programs=6, seed=3))
    X[:, 7] = 0
    X[5, 9] = -1.0
    for M in (X, X + 0.001 * torch.rand_like(X)):
        mn, sq, neg = ops.colstats(M.cuda())
        rmn, rsq, rneg = reference.colstats(M)
        assert torch.equal(mn.cpu(), rmn) and torch.equal(neg.cpu(), rneg)
        np.testing.assert_allclose(sq.cpu().numpy(), rsq.numpy(), rtol=1e-12)
        fmn = torch.where(torch.isfinite(rmn), rmn, torch.ones_like(rmn))
        assert torch.equal(ops.count_unit_check(M.cuda(), fmn.cuda()).cpu(),
                           reference.count_unit_check(M, fmn))


@pytest.mark.parametrize("algo", ["mu", "hals"])
@pytest.mark.parametrize("K", [40, 48, 64])
@pytest.mark.parametrize("conv_mode", [0, 1])
def test_solve_wide_k_matches_fp64_reference(algo, K, conv_mode):
    """Wide ranks (the padded K in (32, 64]) on the 256-thread streaming instantiations."""
    x0, numer, gram = _problem(3, K, 3000, seed=K)
    xg = x0.clone().cuda()
    it_g = torch.zeros(3, dtype=torch.int32, device="cuda")
    ops.solve(algo, xg, numer.cuda(), gram.cuda(), max_iter=40, tol=1e-3, conv_mode=conv_mode,
              iters_out=it_g)
    xr = x0.double().clone()
    it_r = torch.zeros(3, dtype=torch.int32)
    ops.solve(algo, xr, numer.double(), gram.double(), max_iter=40, tol=1e-3,
              conv_mode=conv_mode, iters_out=it_r)
    assert (it_g.cpu() - it_r).abs().max() <= 1
    np.testing.assert_allclose(xg.cpu().double().numpy(), xr.numpy(), rtol=2e-3, atol=1e-4)


@pytest.mark.parametrize("K", [33, 40, 64])
def test_gram_wide_k_matches_bmm(K):
    X = torch.rand((5, K, 3001), dtype=torch.float32)
    out = ops.gram(X.cuda())
    ref = torch.bmm(X.double(), X.double().transpose(1, 2))
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), rtol=1e-5)


@pytest.mark.parametrize("K", [80, 96, 128])
@pytest.mark.parametrize("conv_mode", [0, 1])
@pytest.mark.parametrize("split", ["none", "coop", "nsplit"])
@pytest.mark.parametrize("variant", ["auto", "stream"])
def test_solve_wmfma_matches_fp64_reference(K, conv_mode, split, variant):
    """K in (64, 128]: the matrix-core wide MU solve (solve_wmfma.hip) against the fp64
    torch reference of the same op, with l1/l2 terms, lin/quad epilogue and iteration
    counts; cooperative slices and the fixed-step column split too.  variant 'auto' =
    split-bf16 Gram apply at K = 96 / 128 (fp32 MFMA at 80), 'stream' = fp32 MFMA."""
    R, n = 3, 2999
    x0, numer, gram = _problem(R, K, n, seed=K + conv_mode)
    kw = dict(max_iter=30, tol=1e-3, conv_mode=conv_mode, l1_num=0.01, l2=0.05)
    if split == "nsplit":
        kw.update(max_iter=1, nsplit=3)
    xg = x0.clone().cuda()
    it_g = torch.zeros(R, dtype=torch.int32, device="cuda")
    lin_g = torch.zeros(R, dtype=torch.float32, device="cuda")
    quad_g = torch.zeros(R, dtype=torch.float32, device="cuda")
    ops.solve("mu", xg, numer.cuda(), gram.cuda(), iters_out=it_g, lin_out=lin_g,
              quad_out=quad_g, coop=3 if split == "coop" else 1, variant=variant, **kw)
    ops.coop_check(xg.device)
    xr = x0.double().clone()
    it_r = torch.zeros(R, dtype=torch.int32)
    lin_r = torch.zeros(R, dtype=torch.float64)
    quad_r = torch.zeros(R, dtype=torch.float64)
    ops.solve("mu", xr, numer.double(), gram.double(), iters_out=it_r, lin_out=lin_r,
              quad_out=quad_r, **kw)
    assert (it_g.cpu() - it_r).abs().max() <= 1
    np.testing.assert_allclose(xg.cpu().double().numpy(), xr.numpy(), rtol=2e-3, atol=1e-4)
    np.testing.assert_allclose(lin_g.cpu().double().numpy(), lin_r.numpy(), rtol=2e-3)
    np.testing.assert_allclose(quad_g.cpu().double().numpy(), quad_r.numpy(), rtol=2e-3)


def test_solve_wmfma_planes_and_rep_index():
    """Wide solve: bf16-planes epilogue equals the split of the result; rep_index/active
    gating leaves inactive replicates untouched."""
    K, R, n = 96, 4, 1500
    x0, numer, gram = _problem(R, K, n, seed=5)
    xg = x0.clone().cuda()
    planes = torch.zeros((3, R * K, n + 12), dtype=torch.int16, device="cuda")
    active = torch.tensor([1, 0, 1, 1], dtype=torch.int32, device="cuda")
    ri = torch.tensor([3, 1, 0], dtype=torch.int32, device="cuda")
    ops.solve("mu", xg, numer.cuda(), gram.cuda(), max_iter=10, tol=0.0, rep_index=ri,
              active=active, planes=planes)
    xr = x0.double().clone()
    ops.solve("mu", xr, numer.double(), gram.double(), max_iter=10, tol=0.0)
    got = xg.cpu().double().numpy()
    np.testing.assert_array_equal(got[1], x0[1].double().numpy())     # inactive
    np.testing.assert_array_equal(got[2], x0[2].double().numpy())     # not in rep_index
    for r in (0, 3):
        np.testing.assert_allclose(got[r], xr[r].numpy(), rtol=2e-3, atol=1e-4)
        ref = torch.zeros((3, K, n + 12), dtype=torch.int16)
        ops.split_planes(xg[r].cpu(), ref)
        np.testing.assert_array_equal(planes[:, r * K:(r + 1) * K].cpu().numpy(), ref.numpy())


def test_hals_beyond_64_takes_the_rank_general_solve():
    """HALS at K > 64 (no tiled instantiation) runs solve_any.hip's Gauss-Seidel sweep and
    matches the reference; past its LDS bound (512) the op raises instead of guessing."""
    from cnmf_torch_amd.ops import reference

    x0, numer, gram = _problem(2, 80, 100)
    assert ops.solve_any_k(ops.ALGOS["hals"], 80)
    xg = x0.cuda()
    ops.solve("hals", xg, numer.cuda(), gram.cuda(), max_iter=3)
    xr = x0.double()
    reference.solve(ops.ALGOS["hals"], xr, numer.double(), gram.double(), None, 3, -1.0, 0.0,
                    0.0, 0.0, 1e-16, None, None, None)
    np.testing.assert_allclose(xg.cpu().double().numpy(), xr.numpy(), rtol=2e-3, atol=1e-5)
    big = torch.rand((1, 520, 64), device="cuda")
    with pytest.raises(ValueError, match="rank-general kernel's maximum 512"):
        ops.solve("hals", big, big.clone(), torch.eye(520, device="cuda")[None].contiguous(),
                  max_iter=1)
    with pytest.raises(ValueError, match="rank-general solve"):
        ops.solve("mu", torch.rand((1, 200, 64), device="cuda"),
                  torch.rand((1, 200, 64), device="cuda"),
                  torch.eye(200, device="cuda")[None].contiguous(), variant="mfma")


@pytest.mark.parametrize("K", [65, 100, 128])
def test_gram_wmfma_k_matches_bmm(K):
    """K in (64, 128]: four 64 x 64 blocks per replicate; also the column-split partials
    (few replicates) and accumulate."""
    for R in (2, 70):
        X = torch.rand((R, K, 2001), dtype=torch.float32)
        base = torch.rand((R, K, K), dtype=torch.float32)
        out = base.cuda()
        ops.gram(X.cuda(), out=out, accumulate=True)
        ref = base.double() + torch.bmm(X.double(), X.double().transpose(1, 2))
        np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), rtol=1e-5)


@pytest.mark.parametrize("K", [70, 128])
def test_nmf_wmfma_k_gpu_matches_cpu(K):
    """K > 64: padded to a multiple of 16 (zero components) on the matrix-core wide solve;
    same factorisation as the CPU oracle at the true K, online and batch."""
    from cnmf_torch_amd.models.nmf import run_nmf_batch

    rs = np.random.default_rng(K)
    N, G = 1500, 400
    X = (rs.gamma(1, 1, (N, 20)) @ rs.gamma(0.5, 1, (20, G)) + 0.1 * rs.random((N, G))).astype(
        np.float32)
    for kw in (dict(online_chunk_size=700, online_max_pass=4),
               dict(mode="batch", batch_max_iter=40)):
        g = run_nmf_batch(X, K, [3, 4], device="cuda", **kw)
        c = run_nmf_batch(X, K, [3, 4], device="cpu", **kw)
        assert g.W.shape == (2 * K, G) and g.HT.shape == (2 * K, N)
        np.testing.assert_allclose(g.err, c.err, rtol=1e-3)
        Wg, Wc = g.W.cpu().numpy(), c.W.cpu().numpy()
        cos = (Wg * Wc).sum(1) / (np.linalg.norm(Wg, axis=1) * np.linalg.norm(Wc, axis=1) + 1e-30)
        assert np.median(cos) > 0.99, np.sort(cos)[:5]


def test_refit_wide_and_unpadded_k_on_gpu():
    """fit_H_online / fit_spectra_online at ranks without their own instantiation (K = 37,
    90) pad with zero components on the GPU and match the CPU refit."""
    from cnmf_torch_amd.models.refit import fit_H_online, fit_spectra_online

    rs = np.random.default_rng(0)
    for K in (37, 90):
        X = rs.random((900, 300)).astype(np.float32)
        W = rs.random((K, 300)).astype(np.float32)
        hg = fit_H_online(X, W, device="cuda", chunk_max_iter=30)
        hc = fit_H_online(X, W, device="cpu", chunk_max_iter=30)
        np.testing.assert_allclose(hg, hc, rtol=5e-3, atol=1e-5)
        sg = fit_spectra_online(X, hc, device="cuda", chunk_max_iter=30)
        sc = fit_spectra_online(X, hc, device="cpu", chunk_max_iter=30)
        np.testing.assert_allclose(sg, sc, rtol=5e-3, atol=1e-5)


def test_solve_at_uninstantiated_k_runs_the_rank_general_solve():
    """A rank without a tiled instantiation (K = 37; the engine pads it, a direct caller
    need not) runs solve_any.hip, never an eager fallback, and matches the reference."""
    from cnmf_torch_amd.ops import reference

    x0, numer, gram = _problem(2, 37, 100)
    assert ops.solve_any_k(ops.ALGOS["mu"], 37)
    xg = x0.cuda()
    ops.solve("mu", xg, numer.cuda(), gram.cuda(), max_iter=2)
    xr = x0.double()
    reference.solve(ops.ALGOS["mu"], xr, numer.double(), gram.double(), None, 2, -1.0, 0.0,
                    0.0, 0.0, 1e-16, None, None, None)
    np.testing.assert_allclose(xg.cpu().double().numpy(), xr.numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("K", [37, 64])
def test_nmf_wide_k_gpu_matches_cpu(K):
    """K > 32: padded to a multiple of 8 on the GPU (zero components), same factorisation
    as the CPU oracle at the true K.  Fixed sweep and pass counts (no tolerance-driven
    stop that a rounding difference could flip), so the two runs do the same updates and
    differ by fp32 reassociation only."""
    from cnmf_torch_amd.models.nmf import run_nmf_batch

    rs = np.random.default_rng(K)
    N, G = 1200, 300
    X = (rs.gamma(1, 1, (N, 12)) @ rs.gamma(0.5, 1, (12, G)) + 0.1 * rs.random((N, G))).astype(
        np.float32)
    kw = dict(online_chunk_size=600, online_max_pass=4, online_h_tol=-1.0, online_w_tol=-1.0,
              online_chunk_max_iter=15, tol=-1.0)
    g = run_nmf_batch(X, K, [3, 4], device="cuda", **kw)
    c = run_nmf_batch(X, K, [3, 4], device="cpu", **kw)
    assert g.W.shape == (2 * K, G) and g.HT.shape == (2 * K, N)
    np.testing.assert_array_equal(g.n_iter, c.n_iter)
    np.testing.assert_allclose(g.err, c.err, rtol=3e-3)
    Wg, Wc = g.W.cpu().numpy(), c.W.cpu().numpy()
    cos = (Wg * Wc).sum(1) / (np.linalg.norm(Wg, axis=1) * np.linalg.norm(Wc, axis=1) + 1e-30)
    assert np.median(cos) > 0.999, np.sort(cos)[:5]


def test_device_kmeans_inertia_matches_sklearn_over_seeds():
    """The default GPU k-means (batched k-means++ + batched Lloyd) reaches sklearn's
    KMeans(n_init=10) inertia on replicate-spectra-like data (consensus clustering)."""
    from sklearn.cluster import KMeans

    from cnmf_torch_amd.models.consensus import kmeans

    worse = 0
    ratios = []
    for seed in range(20):
        rs = np.random.default_rng(seed)
        k, reps, G = 7, 40, 300
        centers = rs.gamma(0.5, 1, (k, G))
        S = np.concatenate([c * rs.lognormal(0, 0.15, (reps, G)) for c in centers])
        S /= np.linalg.norm(S, axis=1, keepdims=True)
        lab = kmeans(torch.from_numpy(S).cuda(), k, n_init=10, random_state=1, backend="device")

        def inertia(lb):
            return sum(((S[lb == c] - S[lb == c].mean(0)) ** 2).sum() for c in np.unique(lb))
        ref = KMeans(n_clusters=k, n_init=10, random_state=1).fit(S).labels_
        r = inertia(lab) / inertia(ref)
        ratios.append(r)
        worse += r > 1 + 1e-9
    assert worse <= 1 and np.mean(ratios) <= 1 + 1e-6, ratios


def test_cluster_medians_device_matches_pandas():
    import pandas as pd

    from cnmf_torch_amd.models.consensus import cluster_medians

    rs = np.random.default_rng(1)
    S = rs.random((301, 123))
    S /= np.linalg.norm(S, axis=1, keepdims=True)
    lab = rs.integers(1, 9, 301)
    got = cluster_medians(torch.from_numpy(S).cuda(), lab, sorted(set(lab))).cpu().numpy()
    ref = pd.DataFrame(S).groupby(lab).median()
    ref = ref.div(ref.sum(axis=1), axis=0).values
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("coop,nsplit", [(1, 1), ("auto", 1), (1, 3)])
@pytest.mark.parametrize("K", [6, 10, 40])
def test_solve_planes_epilogue_equals_split_of_result(coop, nsplit, K):
    """The solve epilogue's bf16 planes (fused A-operand split for the next GEMM) are
    bit-identical to ops.split_planes of the final x, times the column multiplier, with
    the k padding zeroed."""
    R, n = 4, 5000
    x0, numer, gram = _problem(R, K, n, seed=K + 7)
    x = x0.clone().cuda()
    pad = -(-n // 32) * 32 + 32
    planes = torch.full((3, R * K, pad), 77, dtype=torch.int16, device="cuda")
    colmul = (torch.rand(n) + 0.5).cuda()
    kw = dict(max_iter=1 if nsplit > 1 else 30, tol=-1.0 if nsplit > 1 else 1e-3,
              nsplit=nsplit, coop=coop)
    ops.solve("mu", x, numer.cuda(), gram.cuda(), planes=planes, planes_colmul=colmul, **kw)
    ref = torch.zeros((3, R * K, pad), dtype=torch.int16, device="cuda")
    ops.split_planes(x.reshape(R * K, n), ref, col_mul=colmul)
    assert torch.equal(planes, ref)


@pytest.mark.parametrize("K", [1, 3, 4, 5, 8, 10, 12, 13, 16])
@pytest.mark.parametrize("conv_mode", [0, 1])
def test_solve_mfma_variant_matches_reference(K, conv_mode):
    """Matrix-core MU solve (solve_mfma.hip: Gram x on v_mfma_f32_16x16x4_f32 with the
    permuted-Gram layout) == the VALU kernel == the fp64 reference: fixed steps with
    l1/l2 penalties and a shifted numerator, then converged solves with cooperative
    slices, lin/quad and iteration counts."""
    R, n = 7, 2500
    x0, numer, gram = _problem(R, K, n, seed=30 + K)
    dev = torch.device("cuda")
    numer_d, gram_d = numer.to(dev), gram.to(dev)
    kw = dict(l1_num=0.01, l1_den=0.02, l2=0.03)
    outs = {}
    for variant in ("mfma", "stream"):
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        ops.solve("mu", xg, numer_d, gram_d, max_iter=6, tol=-1.0, lin_out=lin, quad_out=quad,
                  iters_out=it, conv_mode=conv_mode, check_every=4, variant=variant, **kw)
        outs[variant] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu())
    xr = x0.clone().double()
    lr = torch.zeros(R, dtype=torch.float64)
    qr = torch.zeros(R, dtype=torch.float64)
    reference.solve(0, xr, numer.double(), gram.double(), None, 6, -1.0, kw["l1_num"],
                    kw["l1_den"], kw["l2"], 1e-16, lr, qr, None, 1, conv_mode, 4)
    xm, lm, qm, im = outs["mfma"]
    assert im.tolist() == [6] * R
    torch.testing.assert_close(xm.double(), xr, rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(xm, outs["stream"][0], rtol=2e-4, atol=1e-5)
    torch.testing.assert_close(lm.double(), lr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(qm.double(), qr, rtol=1e-4, atol=1e-3)
    # converged, cooperative slices picked by the host (S > 1 at this n for every K)
    res = {}
    for variant in ("mfma", "stream"):
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        ops.solve("mu", xg, numer_d, gram_d, max_iter=300, tol=1e-4, lin_out=lin,
                  quad_out=quad, iters_out=it, conv_mode=conv_mode, check_every=5,
                  variant=variant)
        res[variant] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu())
    ops.coop_check(dev)
    xm, lm, qm, im = res["mfma"]
    xs, ls, qs, is_ = res["stream"]
    # the objective checks round differently (MFMA vs fmaf chains): a replicate may stop
    # one check later (5 steps), which moves a still-converging x by up to ~0.5 %
    assert (im - is_).abs().max() <= 5
    assert ((xm - xs).norm() / xs.norm()) < 1e-2
    torch.testing.assert_close(lm, ls, rtol=2e-3, atol=1e-3)
    torch.testing.assert_close(qm, qs, rtol=2e-3, atol=1e-3)


def test_solve_mfma_rep_index_active_and_nsplit():
    """Matrix-core solve: untouched replicates stay bit-identical, and the fixed-step
    column split (batch mode, atomically summed lin/quad) == the reference."""
    R, K, n = 8, 11, 3000
    x0, numer, gram = _problem(R, K, n, seed=9)
    dev = torch.device("cuda")
    active = torch.tensor([1, 0, 1, 1, 0, 1, 1, 1], dtype=torch.int32, device=dev)
    ri = torch.tensor([0, 1, 2, 5, 7], dtype=torch.int32, device=dev)
    xg = x0.clone().to(dev)
    ops.solve("mu", xg, numer.to(dev), gram.to(dev), rep_index=ri, max_iter=5, tol=-1.0,
              active=active, variant="mfma")
    xg = xg.cpu()
    for r in (1, 3, 4, 6):
        assert torch.equal(xg[r], x0[r])
    xr = x0.clone().double()
    reference.solve(0, xr, numer.double(), gram.double(), None, 5, -1.0, 0, 0, 0, 1e-16,
                    None, None, None)
    for r in (0, 2, 5, 7):
        torch.testing.assert_close(xg[r].double(), xr[r], rtol=2e-4, atol=1e-5)
    xg = x0.clone().to(dev)
    lin = torch.zeros(R, device=dev)
    quad = torch.zeros(R, device=dev)
    ops.solve("mu", xg, numer.to(dev), gram.to(dev), max_iter=1, nsplit=5, lin_out=lin,
              quad_out=quad, variant="mfma")
    xr = x0.clone().double()
    lr = torch.zeros(R, dtype=torch.float64)
    qr = torch.zeros(R, dtype=torch.float64)
    reference.solve(0, xr, numer.double(), gram.double(), None, 1, -1.0, 0, 0, 0, 1e-16, lr, qr,
                    None)
    torch.testing.assert_close(xg.cpu().double(), xr, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(lin.cpu().double(), lr, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(quad.cpu().double(), qr, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 2000, 5024), (1000, 5000, 2016), (300, 700, 1024)])
def test_gemm_two_a_planes_within_fp32_library_error(M, N, K):
    """Two A planes (hi + mid, <= 2^-16 relative each, ops.gemm_a_planes) against integer
    counts: the product's error vs fp64 is no larger than the fp32 library GEMM's
    (hipBLASLt through torch.matmul) on the same fp32 operands, at the engine's shapes."""
    g = torch.Generator().manual_seed(M + K)
    A = torch.rand((M, K), generator=g) * torch.rand((M, 1), generator=g) * 3
    B = torch.randint(0, 60, (N, K), generator=g).float() * (torch.rand((N, K), generator=g) < 0.3)
    bk = ops.planes_bk(1)
    Kd = -(-K // bk) * bk
    Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device="cuda")
    Bp = torch.zeros((1, N, Kd), dtype=torch.int16, device="cuda")
    ops.split_planes(A.cuda(), Ap)
    ops.split_planes(B.cuda(), Bp)
    ref = A.double() @ B.double().t()
    scale = ref.abs().max()
    C2 = torch.empty((M, N), device="cuda")
    ops.gemm_planes(C2, Ap[:2], Bp, M, N, Kd)
    C3 = torch.empty((M, N), device="cuda")
    ops.gemm_planes(C3, Ap, Bp, M, N, Kd)
    lib = A.cuda() @ B.cuda().t()
    e2 = float((C2.cpu().double() - ref).abs().max() / scale)
    e3 = float((C3.cpu().double() - ref).abs().max() / scale)
    el = float((lib.cpu().double() - ref).abs().max() / scale)
    assert e3 <= e2 * 1.5 + 1e-9
    assert e2 <= max(el, 2e-7), (e2, e3, el)


@pytest.mark.parametrize("K,m", [(3, 2000), (10, 2000), (10, 1997), (16, 333), (20, 2000)])
def test_solve_gram_of_matches_explicit_gram(K, m):
    """ops.solve(gram_of=F): the matrix-core kernel forms F F^T in its prologue (K <= 16;
    unaligned widths take the scalar loads), the VALU kernels get ops.gram's -- same
    iterates as passing the explicit Gram, fixed steps and converged cooperative solves,
    untouched inactive replicates."""
    R, n = 6, 2600
    g = torch.Generator().manual_seed(K + m)
    dev = torch.device("cuda")
    F = (torch.rand((R, K, m + 3), generator=g) + 0.05).to(dev)[:, :, 1:m + 1]  # strided
    gram = torch.bmm(F.double(), F.transpose(1, 2).double()).float()
    x0 = torch.rand((R, K, n), generator=g) + 0.1
    numer = (torch.bmm(gram.cpu(), torch.rand((R, K, n), generator=g))).to(dev)
    active = torch.tensor([1, 1, 0, 1, 1, 1], dtype=torch.int32, device=dev)
    for max_iter, tol, cm in ((6, -1.0, 0), (300, 1e-4, 1)):
        outs = []
        for use_of in (False, True):
            xg = x0.clone().to(dev)
            lin = torch.zeros(R, device=dev)
            it = torch.zeros(R, dtype=torch.int32, device=dev)
            ops.solve("mu", xg, numer, None if use_of else gram, max_iter=max_iter, tol=tol,
                      conv_mode=cm, check_every=5, lin_out=lin, iters_out=it, active=active,
                      gram_of=F if use_of else None)
            outs.append((xg.cpu(), lin.cpu(), it.cpu()))
        (xa, la, ia), (xb, lb, ib) = outs
        torch.testing.assert_close(xb, xa, rtol=2e-5, atol=1e-6)
        torch.testing.assert_close(lb, la, rtol=2e-5, atol=1e-4)
        assert (ib - ia).abs().max() <= (0 if tol < 0 else 5)
        assert torch.equal(xb[2], x0[2])


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("bk,stages", [(32, 2), (32, 3), (64, 2)])
def test_gemm_planes_every_tile_variant(monkeypatch, variant, bk, stages):
    """Every tile variant (incl. the 4-wave 64 x 128 tile of 32 x 64 wave blocks), k-step
    depth and LDS stage count, with and without a k split, == the fp64 product."""
    M, N, K, pb = 301, 650, 1000, 1
    g = torch.Generator().manual_seed(variant * 7 + bk + stages)
    Kd = -(-K // ops.planes_bk(pb)) * ops.planes_bk(pb)
    A = torch.rand((M, K), generator=g)
    B = torch.randint(0, 200, (N, K), generator=g).float()
    Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device="cuda")
    Bp = torch.zeros((pb, N, Kd), dtype=torch.int16, device="cuda")
    ops.split_planes(A.cuda(), Ap)
    ops.split_planes(B.cuda(), Bp)
    ref = A.double() @ B.double().t()
    for ks in (1, 3):
        for k, v in (("CNMF_GEMM_VARIANT", variant), ("CNMF_GEMM_KSPLIT", ks),
                     ("CNMF_GEMM_BK", bk), ("CNMF_GEMM_STAGES", stages)):
            monkeypatch.setenv(k, str(v))
        ops.refresh_env()
        C = torch.empty((M, N), device="cuda")
        ops.gemm_planes(C, Ap, Bp, M, N, Kd)
        torch.cuda.synchronize()
        err = float((C.cpu().double() - ref).abs().max() / ref.abs().max())
        assert err < 1e-6 * K / 256, (variant, bk, stages, ks, err)
    monkeypatch.undo()
    ops.refresh_env()


@pytest.mark.parametrize("K", [1, 3, 5, 10, 12, 13, 16])
@pytest.mark.parametrize("n,coop", [(500, 1), (3100, "auto"), (5000, "auto")])
def test_solve_pipe_bitwise_equals_mfma_kernel(monkeypatch, K, n, coop):
    """The software-pipelined matrix-core MU solve (solve_pipe.hip: compile-time tile
    count, chain(i + 1) issued before the update of tile i, planes from registers) does
    the SAME fp32 operations in the same order as solve_mfma_kernel: converged solves
    (block objective, cooperative slices, an inactive replicate, rep_index) agree
    bitwise in x, lin/quad, iteration counts and the emitted planes -- and the two
    planes it writes are the first two of ops.split_planes of the result."""
    R = 6
    x0, numer, gram = _problem(R, K, n, seed=50 + K)
    dev = torch.device("cuda")
    numer_d, gram_d = numer.to(dev), gram.to(dev)
    active = torch.tensor([1, 1, 0, 1, 1, 1], dtype=torch.int32, device=dev)
    ri = torch.tensor([0, 2, 3, 5], dtype=torch.int32, device=dev)
    pad = -(-n // 64) * 64 + 64
    out = {}
    for pipe in ("1", "0"):
        monkeypatch.setenv("CNMF_SOLVE_PIPE", pipe)
        ops.refresh_env()
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        planes = torch.full((3, R * K, pad), 77, dtype=torch.int16, device=dev)
        ops.solve("mu", xg, numer_d, gram_d, rep_index=ri, max_iter=200, tol=1e-4,
                  lin_out=lin, quad_out=quad, iters_out=it, conv_mode=1, check_every=4,
                  active=active, coop=coop, planes=planes, planes_n=2)
        out[pipe] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu(), planes.cpu())
    monkeypatch.delenv("CNMF_SOLVE_PIPE")
    ops.refresh_env()
    ops.coop_check(dev)
    for a, b in zip(out["1"], out["0"]):
        assert torch.equal(a, b)
    xp, _, _, itp, plp = out["1"]
    assert itp[1].item() == 0 and itp[4].item() == 0 and itp[2].item() == 0  # untouched
    assert torch.equal(xp[2], x0[2]) and torch.equal(xp[1], x0[1])
    assert (itp[[0, 3, 5]] > 0).all()
    ref = torch.zeros((3, R * K, pad), dtype=torch.int16, device=dev)
    ops.split_planes(xp.to(dev).reshape(R * K, n), ref)
    for r in (0, 3, 5):
        rows = slice(r * K, (r + 1) * K)
        assert torch.equal(plp[:2, rows], ref[:2, rows].cpu())
        assert (plp[2, rows] == 77).all()          # the third plane is never written
    # and against the fp64 reference solve of the same stopping rule
    xr = x0.clone().double()
    reference.solve(0, xr, numer.double(), gram.double(), None, 200, 1e-4, 0, 0, 0, 1e-16,
                    None, None, None, 1, 1, 4)
    for r in (0, 3, 5):
        assert ((xp[r].double() - xr[r]).norm() / xr[r].norm()) < 1e-2


@pytest.mark.parametrize("ks", [[10], [5, 7, 13]])
def test_fused_online_step_matches_unfused(monkeypatch, ks):
    """The fused online step (raw split-K slabs summed by the pipelined solves, Grams
    handed between the solves as per-slice partials -- no gemm_reduce / gram launches)
    factorises like the unfused step: same pass counts (+-1), errors to 1e-5, spectra to
    fp32 rounding of a converged iteration."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=8, seed=5)).cuda()
    seeds = list(range(101, 101 + 12 * len(ks)))
    kk = [k for k in ks for _ in range(12)]
    opts = dict(n_components=ks[0], online_chunk_size=2000, online_chunk_max_iter=1000)
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CNMF_FUSED_STEP", fused)
        solver = NMFBatchSolver(X, NMFOptions(**opts))
        if fused == "1":
            from cnmf_torch_amd.models.nmf import _Batch
            st = _Batch(torch.zeros((sum(kk), 6000), device="cuda"),
                        torch.zeros((sum(kk), 700), device="cuda"), sorted(kk))
            assert solver._fused_ok(st, solver._steps(6000))
        out[fused] = solver.run(seeds, ks=kk)
    a, b = out["1"], out["0"]
    assert np.abs(a.n_iter - b.n_iter).max() <= 1
    same = a.n_iter == b.n_iter
    assert same.mean() > 0.8
    np.testing.assert_allclose(a.err[same], b.err[same], rtol=1e-5)
    for r in np.flatnonzero(same):
        wa, wb = a.spectra(r).cpu(), b.spectra(r).cpu()
        assert float((wa - wb).norm() / wb.norm()) < 1e-3


def test_fused_graph_replay_across_runs_is_bitwise_eager(monkeypatch):
    """Fused online passes replayed from the per-layout HIP graphs (captured once, kept
    across runs in the solver's arena) give bit-identical factorisations to the eager
    fused passes, run after run (the second and third runs replay graphs captured in
    the first), and the arena keeps the same buffers."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(5000, 600, n_programs=6, seed=8)).cuda()
    opts = NMFOptions(n_components=6, online_chunk_size=2000, online_chunk_max_iter=1000)
    batches = [list(range(1 + 40 * i, 41 + 40 * i)) for i in range(3)]
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("CNMF_GRAPHS", mode)
        solver = NMFBatchSolver(X, opts)
        res[mode] = [solver.run(b) for b in batches]
        if mode == "1":
            arenas = list(solver._arenas.values())
            assert len(arenas) == 1
            slots = arenas[0]["slots"]
            assert any(sl["graph"] is not None for sl in slots.values())
            assert not any(sl["failed"] for sl in slots.values())
            # replays tag their cooperative exchanges from the device-side generation,
            # which keeps advancing: the workspace was reserved before capture, so no
            # zero-fill / reset of it was recorded into the graphs
            for sl in slots.values():
                if sl["graph"] is not None:
                    ws = ops._COOP_WS[(str(X.device), sl["stream"].cuda_stream)]
                    gen = int(ws["gen_dev"].item()) & 0xFFFFFFFF
                    assert gen > 0x80000000 + 4, hex(gen)
    for a, b in zip(res["1"], res["0"]):
        np.testing.assert_array_equal(a.n_iter, b.n_iter)
        np.testing.assert_array_equal(a.err, b.err)
        assert torch.equal(a.W, b.W) and torch.equal(a.HT, b.HT)


@pytest.mark.parametrize("coop_gen", [False, True])
def test_solve_fused_operands_bitwise(coop_gen):
    """Fused operands of the pipelined solve: numer = base + scale * (sum of raw split-K
    slabs) and Gram = base + sum of partial Grams reproduce, bit for bit, the same solve
    fed the explicitly reduced operands (summed in the same order); numer_out / gram_out
    receive those sums; gram_parts_out holds per-slice partial Grams of the final x."""
    R, K, n, ns, npart = 5, 10, 3000, 3, 7
    x0, numer, gram = _problem(R, K, n, seed=77)
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    slabs = (torch.rand((ns, R, K, n), generator=g) * numer.unsqueeze(0) / ns).to(dev)
    scale = (torch.rand(n, generator=g) + 0.5).to(dev)
    base = (torch.rand((R, K, n), generator=g) * numer.mean()).to(dev)
    parts = (torch.rand((R, npart, K, K), generator=g) * gram.unsqueeze(1) / npart).to(dev)
    gbase = (gram * 0.1).to(dev)
    nref = slabs[0].clone()
    for q in range(1, ns):
        nref = nref + slabs[q]
    nref = base + nref * scale
    t = parts[:, 0].clone()
    for q in range(1, npart):
        t = t + parts[:, q]
    gref = gbase + t
    kw = dict(max_iter=300, tol=1e-4, conv_mode=1, check_every=5)
    x1 = x0.clone().to(dev)
    S1 = ops.solve("mu", x1, nref, gref, **kw)
    x2 = x0.clone().to(dev)
    nout = torch.zeros_like(nref)
    gout = torch.zeros_like(gref)
    gp_out = torch.full((R, 32, K, K), float("nan"), device=dev)
    flat = slabs.reshape(-1)
    S2 = ops.solve("mu", x2, flat[:R * K * n].view(R, K, n), gbase, numer_slabs=ns,
                   numer_slab_stride=R * K * n, numer_scale=scale, numer_base=base,
                   numer_out=nout, gram_parts=parts, gram_parts_n=npart, gram_out=gout,
                   gram_parts_out=gp_out, coop_device_gen=coop_gen, **kw)
    ops.coop_check(dev)
    assert S1 == S2 and S2 > 1
    assert torch.equal(x1, x2)
    assert torch.equal(nout, nref) and torch.equal(gout, gref)
    full = torch.bmm(x2.double(), x2.double().transpose(1, 2))
    got = gp_out[:, :S2].double().sum(dim=1)
    torch.testing.assert_close(got, full, rtol=1e-5, atol=1e-6)
    assert torch.isnan(gp_out[:, S2:]).all()


@pytest.mark.parametrize("M,N,K", [(1000, 2000, 5024), (1000, 5000, 2016)])
def test_gemm_two_b_planes_within_fp32_library_error(M, N, K):
    """Non-count data in two B planes (hi + mid; models.nmf._XPlanes._float_planes) times
    two A planes: the product's error vs fp64 is no larger than the fp32 library GEMM's
    on the same operands at the engine's shapes (reduction >= 1024)."""
    g = torch.Generator().manual_seed(M + 3 * K)
    A = torch.rand((M, K), generator=g) * torch.rand((M, 1), generator=g) * 3
    B = torch.rand((N, K), generator=g) * 7 + 0.5
    bk = ops.planes_bk(2)
    Kd = -(-K // bk) * bk
    Ap = torch.zeros((3, M, Kd), dtype=torch.int16, device="cuda")
    Bp = torch.zeros((3, N, Kd), dtype=torch.int16, device="cuda")
    ops.split_planes(A.cuda(), Ap)
    ops.split_planes(B.cuda(), Bp)
    ref = A.double() @ B.double().t()
    scale = ref.abs().max()
    C22 = torch.empty((M, N), device="cuda")
    ops.gemm_planes(C22, Ap[:2], Bp[:2], M, N, Kd)
    lib = A.cuda() @ B.cuda().t()
    e22 = float((C22.cpu().double() - ref).abs().max() / scale)
    el = float((lib.cpu().double() - ref).abs().max() / scale)
    assert e22 <= max(el, 2e-7), (e22, el)


@pytest.mark.parametrize("n,G,k", [(1300, 2000, 10), (57, 33, 1), (4096, 50, 256), (900, 7, 13)])
def test_seg_median_kernel_matches_pandas_with_ties(n, G, k):
    """seg_median.hip (per-gene in-LDS rank counting) == pandas groupby().median(), bit
    for bit, with heavy ties (values on a coarse grid) and odd / even cluster sizes; the
    consensus medians run it (not the sort fallback) up to 4096 spectra."""
    import pandas as pd

    rs = np.random.default_rng(n + k)
    S = np.round(rs.random((n, G)) * 40) / 40.0
    lab = rs.integers(0, k, n)
    lab[:k] = np.arange(k)                      # every cluster non-empty
    St = torch.from_numpy(S).cuda()
    got = ops.seg_median(St, lab, k)
    assert got is not None
    ref = pd.DataFrame(S).groupby(lab).median().values
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    assert ops.seg_median(torch.zeros((4097, 3), dtype=torch.float64, device="cuda"),
                          np.arange(4097) % 3, 3) is None          # beyond the LDS stage


def test_gemm_gate_skips_and_runs():
    """gemm_planes(gate=...): a zero gate leaves the output untouched (every workgroup
    returns once its prologue loads drained; without a k split nothing else runs), a one
    gate computes the product (with and without a k split)."""
    g = torch.Generator().manual_seed(7)
    M, N, Kd = 200, 300, 512
    a = torch.rand((M, Kd), generator=g)
    b = torch.randint(0, 20, (N, Kd), generator=g).float()
    A = torch.zeros((2, M, Kd), dtype=torch.int16, device="cuda")
    B = torch.zeros((1, N, Kd), dtype=torch.int16, device="cuda")
    ops.split_planes(a.cuda(), A)
    ops.split_planes(b.cuda(), B)
    ref = (a.double() @ b.double().t()).numpy()
    for ksplit in ("1", "4"):
        os.environ["CNMF_GEMM_KSPLIT"] = ksplit
        ops.refresh_env()
        try:
            C = torch.full((M, N), -7.0, device="cuda")
            if ksplit == "1":
                ops.gemm_planes(C, A, B, M, N, Kd, gate=torch.zeros(1, dtype=torch.int32,
                                                                      device="cuda"))
                assert bool((C == -7.0).all())
            ops.gemm_planes(C, A, B, M, N, Kd, gate=torch.ones(1, dtype=torch.int32,
                                                                 device="cuda"))
            np.testing.assert_allclose(C.cpu().double().numpy(), ref, rtol=1e-5)
        finally:
            os.environ.pop("CNMF_GEMM_KSPLIT", None)
            ops.refresh_env()


@pytest.mark.parametrize("n,d,k,nr", [(900, 2000, 10, 40), (1234, 333, 7, 3), (64, 70, 200, 2),
                                      (5, 130, 3, 1)])
def test_seg_colsum_matches_float64_reference(n, d, k, nr):
    """segsum.hip seg_colsum (the k-means centroid sums of every restart) == float64
    index_add over the same labels, to 1e-12 relative; deterministic across calls."""
    g = torch.Generator().manual_seed(n + d + k)
    X = torch.rand((n, d), generator=g, dtype=torch.float64)
    lab = torch.randint(0, k, (nr, n), generator=g)
    want = ops.seg_colsum(X, lab, k)                  # CPU: index_add in point order
    got = ops.seg_colsum(X.cuda(), lab.cuda(), k)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-12, atol=1e-12)
    assert torch.equal(got, ops.seg_colsum(X.cuda(), lab.cuda(), k))


@pytest.mark.parametrize("n,m,k", [(1000, 1000, 10), (333, 777, 57), (65, 64, 250)])
def test_seg_rowsum_and_device_silhouette_match_sklearn(n, m, k):
    """segsum.hip seg_rowsum == float64 reference sums; the device silhouette built on
    it == sklearn.metrics.silhouette_score(precomputed) to 1e-10."""
    from sklearn.metrics import silhouette_score

    from cnmf_torch_amd.models.consensus import pairwise_distances, silhouette

    g = torch.Generator().manual_seed(n + m + k)
    D = torch.rand((n, m), generator=g, dtype=torch.float64)
    lab = torch.randint(0, k, (m,), generator=g)
    torch.testing.assert_close(ops.seg_rowsum(D.cuda(), lab.cuda(), k).cpu(),
                               ops.seg_rowsum(D, lab, k), rtol=1e-12, atol=1e-12)
    rs = np.random.default_rng(k)
    X = rs.random((n, 12))
    labs = rs.integers(0, min(k, n // 3), n)
    Dx = pairwise_distances(torch.from_numpy(X).cuda())
    got = silhouette(Dx, labs)
    want = silhouette_score(Dx.cpu().numpy(), labs, metric="precomputed")
    assert abs(got - want) <= 1e-10


@pytest.mark.parametrize("n,K,dt", [(10000, 13, torch.float64), (2000, 9, torch.float32),
                                    (77, 64, torch.float64), (5, 3, torch.float32)])
def test_small_gram_matches_float64(n, K, dt):
    """segsum.hip small_gram_kernel (the consensus / refit / OLS K x K Grams) == the
    float64 product, for A^T A of an (n x K) operand and A A^T of a (K x n) one, strided
    views included; deterministic across calls."""
    g = torch.Generator().manual_seed(n + K)
    A = torch.rand((n, K + 3), generator=g, dtype=torch.float64)[:, 1:K + 1]   # strided
    want = A.t() @ A
    tol = 1e-12 if dt == torch.float64 else 2e-6
    got = ops.small_gram(A.to(dt).cuda())
    torch.testing.assert_close(got.double().cpu(), want, rtol=tol, atol=tol)
    assert torch.equal(got, ops.small_gram(A.to(dt).cuda()))
    B = A.t().contiguous()                                   # (K x n)
    got2 = ops.small_gram(B.to(dt).cuda(), rows_are_points=False)
    torch.testing.assert_close(got2.double().cpu(), want, rtol=tol, atol=tol)

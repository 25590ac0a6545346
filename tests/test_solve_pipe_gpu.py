"""The pipelined matrix-core MU solve at 17 <= K <= 64 (csrc/kernels/solve_pipe.h: MB =
K/16 output blocks of permuted Gram rows, register-resident iterate, co-resident launch
rounds) and the fused online step / per-layout graphs that run on it, against the fp64
reference solve, the VALU kernel, and the unfused / eager paths."""
import os

import numpy as np
import pytest
import torch

from cnmf_torch_amd import ops
from cnmf_torch_amd.ops import reference

pytestmark = pytest.mark.gpu

WIDE_K = [17, 20, 24, 32, 40, 48, 64]


def _problem(R, K, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    W = torch.rand((R, K, 96), generator=g, dtype=torch.float64) + 0.05
    gram = torch.bmm(W, W.transpose(1, 2))
    x_true = torch.rand((R, K, n), generator=g, dtype=torch.float64)
    numer = torch.bmm(gram, x_true) * (1 + 0.05 * torch.rand((R, K, n), generator=g,
                                                             dtype=torch.float64))
    x0 = torch.rand((R, K, n), generator=g, dtype=torch.float64) + 0.1
    return x0.float(), numer.float(), gram.float()


@pytest.mark.parametrize("K", WIDE_K)
def test_solve_pipe_wide_k_matches_reference(K):
    """Fixed steps == the fp64 reference (and the VALU kernel) in x, lin, quad and the
    iteration count; converged cooperative solves agree with the VALU kernel's."""
    R, n = 5, 2600
    x0, numer, gram = _problem(R, K, n, seed=300 + K)
    dev = torch.device("cuda")
    numer_d, gram_d = numer.to(dev), gram.to(dev)
    assert ops.pipe_slices(n, R, K, dev) is not None
    outs = {}
    for variant in ("auto", "stream"):
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        ops.solve("mu", xg, numer_d, gram_d, max_iter=6, tol=-1.0, lin_out=lin, quad_out=quad,
                  iters_out=it, conv_mode=1, check_every=4, variant=variant)
        outs[variant] = (xg.cpu(), lin.cpu(), quad.cpu(), it.cpu())
    xr = x0.clone().double()
    lr = torch.zeros(R, dtype=torch.float64)
    qr = torch.zeros(R, dtype=torch.float64)
    reference.solve(0, xr, numer.double(), gram.double(), None, 6, -1.0, 0.0, 0.0, 0.0, 1e-16,
                    lr, qr, None, 1, 1, 4)
    xm, lm, qm, im = outs["auto"]
    assert im.tolist() == [6] * R
    torch.testing.assert_close(xm.double(), xr, rtol=3e-4, atol=1e-5)
    torch.testing.assert_close(xm, outs["stream"][0], rtol=3e-4, atol=1e-5)
    torch.testing.assert_close(lm.double(), lr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(qm.double(), qr, rtol=1e-4, atol=1e-3)
    res = {}
    for variant in ("auto", "stream"):
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        ops.solve("mu", xg, numer_d, gram_d, max_iter=300, tol=1e-4, lin_out=lin,
                  iters_out=it, conv_mode=1, check_every=5, variant=variant)
        res[variant] = (xg.cpu(), lin.cpu(), it.cpu())
    ops.coop_check(dev)
    (xm, lm, im), (xs, ls, is_) = res["auto"], res["stream"]
    assert (im - is_).abs().max() <= 5
    assert ((xm - xs).norm() / xs.norm()) < 1e-2
    torch.testing.assert_close(lm, ls, rtol=2e-3, atol=1e-3)


@pytest.mark.parametrize("K", [20, 40, 64])
def test_solve_pipe_launch_rounds_bitwise_one_launch(monkeypatch, K):
    """With a small co-residency budget the replicates run in several launch rounds
    (reps_per_launch): same slices, so bit-identical to one launch; an inactive
    replicate and rep_index are honoured across rounds."""
    R, n = 7, 3000
    x0, numer, gram = _problem(R, K, n, seed=400 + K)
    dev = torch.device("cuda")
    numer_d, gram_d = numer.to(dev), gram.to(dev)
    active = torch.tensor([1, 1, 0, 1, 1, 1, 1], dtype=torch.int32, device=dev)
    ri = torch.tensor([0, 1, 2, 4, 5, 6], dtype=torch.int32, device=dev)
    S = 12
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    full = ops._coop_resident(dev)
    out = []
    for resident in (full, 2 * S // ops._hip.solve_pipe_wg_per_cu(K)):
        monkeypatch.setitem(ops._COOP_RESIDENT, key, resident)
        plan = ops._pipe_plan(n, ri.numel(), K, S, dev)
        assert plan is not None and plan[0] == S
        if resident != full:
            assert 0 < plan[1] < ri.numel()      # several rounds
        xg = x0.clone().to(dev)
        lin = torch.zeros(R, device=dev)
        quad = torch.zeros(R, device=dev)
        it = torch.zeros(R, dtype=torch.int32, device=dev)
        got = ops.solve("mu", xg, numer_d, gram_d, rep_index=ri, max_iter=200, tol=1e-4,
                        lin_out=lin, quad_out=quad, iters_out=it, conv_mode=1, check_every=4,
                        active=active, coop=S)
        assert got == S
        out.append((xg.cpu(), lin.cpu(), quad.cpu(), it.cpu()))
    ops.coop_check(dev)
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    xg, _, _, it = out[0]
    assert torch.equal(xg[2], x0[2]) and torch.equal(xg[3], x0[3])
    assert it[2].item() == 0 and it[3].item() == 0 and (it[[0, 1, 4, 5, 6]] > 0).all()


@pytest.mark.parametrize("K", [20, 40])
@pytest.mark.parametrize("coop_gen", [False, True])
def test_solve_pipe_fused_operands_bitwise_wide(K, coop_gen):
    """Fused operands at K > 16 (MB > 1 Gram blocks): raw slabs + scale + base, partial
    Grams + base reproduce the explicitly reduced operands bit for bit; numer_out /
    gram_out get those sums; the per-slice partial Grams (MB x MB 16 x 16 blocks each)
    sum to x x^T."""
    R, n, ns, npart = 5, 3000, 3, 7
    x0, numer, gram = _problem(R, K, n, seed=77 + K)
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
    # every slice's partial is itself symmetric, bit for bit
    p = gp_out[:, :S2]
    assert torch.equal(p, p.transpose(2, 3))
    assert torch.isnan(gp_out[:, S2:]).all()


@pytest.mark.parametrize("ks", [[20], [17, 24, 32], [48], [64]])
def test_fused_online_step_matches_unfused_wide(monkeypatch, ks):
    """The fused online step at K > 16 (the cNMF-typical ranks; K = 48 padded from 41)
    factorises like the unfused step: pass counts +-1, errors to 1e-5, spectra to fp32
    rounding of a converged iteration."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions, _Batch, native_rank
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=12, seed=5)).cuda()
    ks = [41 if k == 48 else k for k in ks]
    seeds = list(range(101, 101 + 10 * len(ks)))
    kk = [k for k in ks for _ in range(10)]
    opts = dict(n_components=ks[0], online_chunk_size=2000, online_chunk_max_iter=1000)
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CNMF_FUSED_STEP", fused)
        solver = NMFBatchSolver(X, NMFOptions(**opts))
        if fused == "1":
            kp = sorted(native_rank(k) for k in kk)
            st = _Batch(torch.zeros((sum(kp), 6000), device="cuda"),
                        torch.zeros((sum(kp), 700), device="cuda"), kp)
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


@pytest.mark.parametrize("K", [20, 33])
def test_fused_graph_replay_wide_k_bitwise_eager(monkeypatch, K):
    """Per-layout HIP-graph replays of the fused passes at K > 16 (K = 33 runs padded to
    40 inside a graph arena) equal the eager passes bit for bit, run after run."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(5000, 600, n_programs=10, seed=8)).cuda()
    opts = NMFOptions(n_components=K, online_chunk_size=2000, online_chunk_max_iter=1000)
    batches = [list(range(1 + 24 * i, 25 + 24 * i)) for i in range(3)]
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
    for a, b in zip(res["1"], res["0"]):
        np.testing.assert_array_equal(a.n_iter, b.n_iter)
        np.testing.assert_array_equal(a.err, b.err)
        assert torch.equal(a.W, b.W) and torch.equal(a.HT, b.HT)
        assert a.W.shape[0] == 24 * K


_COMPACT_CASES = [([10], "0"), ([5, 7, 13], "0"), ([20], "0"), ([5, 7, 13], "1"), ([20], "1")]


def _case_id(ks, pmap):
    return "k" + "_".join(map(str, ks)) + "-map" + pmap


@pytest.mark.parametrize("ks,pmap", [pytest.param(k, m, id=_case_id(k, m))
                                     for k, m in _COMPACT_CASES])
def test_host_compaction_matches_uncompacted(monkeypatch, ks, pmap):
    """Host compaction of finished replicates (in-place row permutation of the arena on
    one-pass-stale flags) changes where rows live, not what is computed: the fused run
    with compaction equals the run that never compacts (finished replicates skipped in
    place) to fp32 rounding -- the compacted GEMMs re-plan their k split."""
    from cnmf_torch_amd.models import nmf
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=10, seed=6)).cuda()
    kk = [k for k in ks for _ in range(14)]
    seeds = list(range(7, 7 + len(kk)))
    opts = nmf.NMFOptions(n_components=ks[0], online_chunk_size=2000,
                          online_chunk_max_iter=1000)
    out = {}
    # (CNMF_PIPE_MAP: the pipelined solve's workgroup order, 1 = XCD-grouped slices; read
    # once per process by the extension, so a case runs in a child process with it set)
    if os.environ.get("CNMF_PIPE_MAP") != pmap:
        import subprocess
        import sys

        env = dict(os.environ, CNMF_PIPE_MAP=pmap)
        r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                            f"{__file__}::test_host_compaction_matches_uncompacted"
                            f"[{_case_id(ks, pmap)}]"], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        return
    for mode in ("plain", "compact"):
        frac = "2.0" if mode == "plain" else "0.25"
        monkeypatch.setenv("CNMF_COMPACT_FRAC", frac)
        monkeypatch.setenv("CNMF_COMPACT_FRAC_SMALL", frac)
        out[mode] = nmf.NMFBatchSolver(X, opts).run(seeds, ks=kk)
    b, c = out["plain"], out["compact"]
    assert len(set(b.n_iter.tolist())) > 1          # replicates finished at different passes
    assert np.abs(b.n_iter - c.n_iter).max() <= 1
    same = b.n_iter == c.n_iter
    assert same.mean() > 0.8
    np.testing.assert_allclose(b.err[same], c.err[same], rtol=1e-5)


def test_rank_beyond_tiled_kernels_runs_native_on_the_gpu(recwarn):
    """K > 128 Frobenius runs the rank-general solve (solve_any.hip) on the GPU -- no eager
    routing, no warning -- and factorises like the CPU engine (same seeds, same algorithm,
    fp32 rounding apart); a mixed batch keeps every K in one ragged batch; refits at that
    rank run natively too."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.models.refit import fit_H_online
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    Xn = normalized_counts_matrix(900, 300, n_programs=6, seed=2)
    opts = NMFOptions(n_components=130, online_chunk_size=450, online_max_pass=4)
    g = NMFBatchSolver(torch.from_numpy(Xn).cuda(), opts).run([5, 6], ks=[130, 10])
    c = NMFBatchSolver(torch.from_numpy(Xn), opts).run([5, 6], ks=[130, 10])
    assert g.W.shape == (140, 300) and torch.isfinite(g.W).all()
    np.testing.assert_allclose(g.err, c.err, rtol=2e-3)
    U = fit_H_online(Xn, g.W[:130].cpu().numpy(), device="cuda")
    assert U.shape == (900, 130) and np.isfinite(U).all() and (U >= 0).all()
    Uc = fit_H_online(Xn, g.W[:130].cpu().numpy(), device="cpu")
    np.testing.assert_allclose(U, Uc, rtol=5e-3, atol=1e-4 * float(np.abs(Uc).max()))
    hals = NMFOptions(n_components=100, algo="hals", online_chunk_size=450, online_max_pass=3)
    gh = NMFBatchSolver(torch.from_numpy(Xn).cuda(), hals).run([3])
    ch = NMFBatchSolver(torch.from_numpy(Xn), hals).run([3])
    np.testing.assert_allclose(gh.err, ch.err, rtol=2e-3)
    assert not [w for w in recwarn.list if "eager" in str(w.message)]


@pytest.mark.gpu
@pytest.mark.parametrize("algo,K,conv,tol", [("mu", 130, 1, 0.0), ("mu", 200, 0, 0.0),
                                              ("mu", 144, 1, 1e-3), ("mu", 136, 0, 1e-3),
                                              ("hals", 80, 1, 0.0), ("hals", 200, 0, 0.0),
                                              ("hals", 72, 1, 1e-3), ("hals", 130, 0, 1e-3)])
def test_solve_any_rank_matches_float64_reference(algo, K, conv, tol):
    """The rank-general solve (ops.solve at K beyond the tiled kernels) == the float64
    reference solve: strided x, a replicate subset (rep_index) with one replicate inactive,
    l1 / l2, both stop rules, lin / quad / iters outputs.  tol = 0 runs every step (x to
    fp32 accuracy, iteration counts exact); tol > 0 stops on the device (counts within one
    check interval, x pinned where the counts agree)."""
    from cnmf_torch_amd import ops
    from cnmf_torch_amd.ops import reference

    g = torch.Generator().manual_seed(K + conv)
    R, n, m = 5, 700, 300
    F = torch.rand((R, K, m), generator=g, dtype=torch.float64)
    gram = torch.bmm(F, F.transpose(1, 2)) / m
    numer = torch.bmm(gram, torch.rand((R, K, n), generator=g, dtype=torch.float64))
    numer *= 0.5 + torch.rand((R, K, n), generator=g, dtype=torch.float64)
    x0 = torch.rand((R, K, n), generator=g, dtype=torch.float64)
    reps = torch.tensor([0, 2, 3, 4], dtype=torch.int32)
    act = torch.tensor([1, 1, 1, 0, 1], dtype=torch.int32)
    kw = dict(max_iter=25, tol=tol, l1_num=1e-3, l1_den=1e-2, l2=2e-2, eps=1e-16,
              conv_mode=conv, check_every=5)
    xr = x0.clone()
    lin_r, quad_r = torch.zeros(R, dtype=torch.float64), torch.zeros(R, dtype=torch.float64)
    it_r = torch.zeros(R, dtype=torch.int32)
    reference.solve(ops.ALGOS[algo], xr, numer, gram, reps, kw["max_iter"], tol, 1e-3, 1e-2,
                    2e-2, 1e-16, lin_r, quad_r, it_r, 1, conv, 5, act)
    buf = torch.zeros((R, K, n + 37), dtype=torch.float32, device="cuda")
    xg = buf[:, :, :n]
    xg.copy_(x0)
    lin_g = torch.zeros(R, dtype=torch.float32, device="cuda")
    quad_g = torch.zeros_like(lin_g)
    it_g = torch.zeros(R, dtype=torch.int32, device="cuda")
    assert ops.solve_any_k(ops.ALGOS[algo], K)
    ops.solve(algo, xg, numer.float().cuda(), gram.float().cuda(), rep_index=reps.cuda(),
              lin_out=lin_g, quad_out=quad_g, iters_out=it_g, active=act.cuda(), **kw)
    torch.cuda.synchronize()
    it_g = it_g.cpu()
    assert it_g[1] == 0 and it_g[3] == 0 and float(lin_g[3]) == 0.0     # untouched
    np.testing.assert_array_equal(xg[3].cpu().numpy(), x0[3].float().numpy())
    if tol == 0.0:
        assert torch.equal(it_g, it_r) and int(it_r[0]) == 25
    else:
        assert (it_g - it_r).abs().max() <= 5
    for r in (0, 2, 4):
        if it_g[r] != it_r[r]:
            continue
        np.testing.assert_allclose(xg[r].cpu().double().numpy(), xr[r].numpy(), rtol=2e-3,
                                   atol=2e-5 * float(xr[r].abs().max()))
        np.testing.assert_allclose(float(lin_g[r]), float(lin_r[r]), rtol=1e-4)
        np.testing.assert_allclose(float(quad_g[r]), float(quad_r[r]), rtol=1e-4)


@pytest.mark.parametrize("N,G,K", [(1000, 300, 10), (777, 2001, 7), (4096, 128, 64), (130, 70, 128)])
def test_predict_err_kernel_matches_float64(N, G, K):
    """predict_err.hip (H8): <X, U S> and ||X||^2 in one pass over the resident float32 X
    with the U S tile on the f64 matrix cores == float64 torch, and the k-selection
    prediction error built from them == ||X - U S||^2 (cnmf.py:1100-1104)."""
    from cnmf_torch_amd.api import cNMF

    g = torch.Generator().manual_seed(N + G + K)
    X = (torch.rand((N, G), generator=g) * (torch.rand((N, G), generator=g) < 0.3)).float()
    U = torch.rand((N, K), generator=g, dtype=torch.float64)
    S = torch.rand((K, G), generator=g, dtype=torch.float64)
    cross, xsq = ops.predict_err_terms(X.cuda(), U, S)
    Xd = X.double()
    want_c = float((Xd * (U @ S)).sum())
    want_x = float((Xd * Xd).sum())
    assert abs(cross - want_c) <= 1e-12 * abs(want_c)
    assert abs(xsq - want_x) <= 1e-12 * abs(want_x)
    err = cNMF._prediction_error(X.cuda(), U.numpy(), S.numpy(), torch.device("cuda"))
    full = float(((Xd - U @ S) ** 2).sum())
    assert abs(err - full) <= 1e-9 * full


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_exact_moments_device_equals_host_digits(dt):
    """exact_moments.hip and the host exact_col_moments produce the SAME integer digits
    (exact sums of x and x^2 per column), so statistics from either -- or from any row
    split of either -- are bit-identical; they equal float64 numpy to rounding."""
    from cnmf_torch_amd.models.hvg import (_digits_to_ints, exact_mean_var,
                                           exact_moment_digits)

    g = torch.Generator().manual_seed(4)
    X = (torch.rand((9000, 333), generator=g) * 50 - 5).to(dt)
    X[X.abs() < 1] = 0
    hd = exact_moment_digits(X.numpy())
    gd = exact_moment_digits(X.cuda())
    assert hd[2] == 0 and gd[2] == 0
    assert _digits_to_ints(hd[0]) == _digits_to_ints(gd[0])
    assert _digits_to_ints(hd[1]) == _digits_to_ints(gd[1])
    m_h, v_h = exact_mean_var(X.numpy(), 1)
    m_g, v_g = exact_mean_var(X.cuda(), 1)
    np.testing.assert_array_equal(m_h, m_g)
    np.testing.assert_array_equal(v_h, v_g)
    Xd = X.double().numpy()
    np.testing.assert_allclose(m_h, Xd.mean(0), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(v_h, Xd.var(0, ddof=1), rtol=1e-10)


@pytest.mark.parametrize("N,F,K,levels", [(5000, 300, 30, (4, 3, 2, 2)), (777, 50, 7, (3,)),
                                          (20000, 70, 100, (6, 4, 3, 2))])
def test_moe_ridge_kernels_match_reference_formula(N, F, K, levels):
    """ridge.hip (level-segment products on the f64 matrix cores, host (B+1)^2 solves,
    combination-grouped correction) == the reference's moe_correct_ridge formula
    (preprocess.py:9-18) in float64 to 1e-10, for the expression matrix (cells x genes)
    and for the PCs inside the Harmony loop; no dense Phi_Rk is formed."""
    from cnmf_torch_amd.models.harmony import (_levels, moe_correct_expression,
                                               moe_correct_ridge, moe_correct_ridge_pcs)

    rs = np.random.default_rng(N + F)
    X = rs.random((N, F)) * 3
    R = rs.random((K, N))
    R /= R.sum(0)
    blocks = []
    for nl in levels:
        b = rs.integers(0, nl, N)
        P = np.zeros((nl, N))
        P[b, np.arange(N)] = 1
        blocks.append(P)
    Phi_moe = np.vstack([np.ones((1, N))] + blocks)
    B1 = Phi_moe.shape[0]
    lamb = np.diag([0.0] + [1.0] * (B1 - 1))
    _, Zc, _, _ = moe_correct_ridge(X.T, None, None, R, None, K, None, Phi_moe, lamb)
    got = moe_correct_expression(torch.from_numpy(X).cuda(), R, Phi_moe, lamb, K=K)
    np.testing.assert_allclose(got.cpu().numpy(), Zc.T, rtol=1e-10, atol=1e-10)
    got32 = moe_correct_expression(torch.from_numpy(X.astype(np.float32)).cuda(), R, Phi_moe,
                                   lamb, K=K)
    assert got32.dtype == torch.float32
    np.testing.assert_allclose(got32.cpu().numpy(), Zc.T.astype(np.float32), rtol=2e-6, atol=2e-6)
    # the PCs path of the Harmony loop (d x N), W included
    lv = _levels(Phi_moe)
    Z = torch.from_numpy(X.T.copy()).cuda()
    Rd, Pd, Ld = (torch.from_numpy(a).cuda() for a in (R, Phi_moe, lamb))
    zc_n, zr_n, w_n = moe_correct_ridge_pcs(Z, Rd, Pd, Ld, levels=lv)
    zc_d, zr_d, w_d = moe_correct_ridge_pcs(Z, Rd, Pd, Ld, levels=None)
    torch.testing.assert_close(zr_n, zr_d, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(zc_n, zc_d, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(w_n, w_d, rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("shape,dt", [((70_000, 300), torch.float32), ((9_000_001,), torch.float64),
                                      ((5, 7), torch.float32)])
def test_to_host_pinned_copy_is_bitwise(shape, dt):
    """utils.transfer.to_host (pinned double-buffered chunks, threaded unpack) returns the
    same bytes as .cpu() for chunk-spanning, odd-sized and small (pageable-path) tensors."""
    from cnmf_torch_amd.utils.transfer import to_host

    t = torch.randn(shape, dtype=dt, device="cuda")
    a = to_host(t, chunk_bytes=16 << 20)
    assert a.dtype == t.cpu().numpy().dtype and a.shape == tuple(shape)
    np.testing.assert_array_equal(a, t.cpu().numpy())
    np.testing.assert_array_equal(to_host(t[1:]), t[1:].cpu().numpy())   # an offset view


@pytest.mark.parametrize("ks", [[10], [5, 7, 13], [20]])
def test_stream_matches_batch_solves(ks):
    """Continuous batching (run_stream: live slots refilled from the queue as replicates
    converge) solves every replicate as the one-batch run does: each its own pass count
    (+-1 where fp32 summation orders of different batch compositions tip a stop test),
    errors of same-pass replicates to 1e-5, and every replicate harvested exactly once
    into the callers' order."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=10, seed=6)).cuda()
    kk = [k for k in ks for _ in range(30)]
    seeds = list(range(101, 101 + len(kk)))
    opts = NMFOptions(n_components=ks[0], online_chunk_size=2000, online_chunk_max_iter=1000)
    solver = NMFBatchSolver(X, opts)
    got = []
    s = solver.run_stream(seeds, ks=kk, live=8,
                          on_result=lambda ids, k_, host, ev: got.extend(ids.tolist()))
    assert s.stats["stream_stagings"] > 0 and s.stats["stream_slots"] == {k: 8 for k in ks}
    assert sorted(got) == list(range(len(kk)))
    b = NMFBatchSolver(X, opts).run(seeds, ks=kk)
    assert (s.ks == b.ks).all()
    assert np.abs(s.n_iter - b.n_iter).max() <= 1
    same = s.n_iter == b.n_iter
    assert same.mean() > 0.8
    np.testing.assert_allclose(s.err[same], b.err[same], rtol=1e-5)
    for r in np.flatnonzero(same)[:20]:
        wa, wb = s.spectra(r).cpu(), b.spectra(r).cpu()
        assert float((wa - wb).norm() / wb.norm()) < 1e-3
        ua, ub = s.usages(r).cpu(), b.usages(r).cpu()
        assert float((ua - ub).norm() / ub.norm()) < 1e-3


def test_stream_graph_replays_bitwise_eager_and_pass_limit(monkeypatch):
    """A streaming run whose passes replay the layout's captured HIP graph (refills are
    written in place between replays) equals the all-eager streaming run bit for bit, and
    the device applies online_max_pass to every replicate separately."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(5000, 600, n_programs=10, seed=8)).cuda()
    opts = NMFOptions(n_components=10, online_chunk_size=2000, online_chunk_max_iter=1000,
                      online_max_pass=6)
    seeds = list(range(3, 3 + 48))
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("CNMF_GRAPHS", mode)
        solver = NMFBatchSolver(X, opts)
        res[mode] = solver.run_stream(seeds, live=16)
        assert res[mode].stats["stream_stagings"] > 0
        if mode == "1":
            slots = list(solver._arenas.values())[0]["slots"]
            assert any(sl["graph"] is not None for sl in slots.values()), \
                [sl.get("error") for sl in slots.values()]
    a, b = res["1"], res["0"]
    np.testing.assert_array_equal(a.n_iter, b.n_iter)
    np.testing.assert_array_equal(a.err, b.err)
    assert torch.equal(a.W, b.W) and torch.equal(a.HT, b.HT)
    assert a.n_iter.max() == 6 and a.n_iter.min() >= 1
    assert np.isfinite(a.err).all() and bool((a.W >= 0).all())


def test_rows_swap_kernel_matches_reference():
    """stream.hip rows_swap_kernel (in-place compaction swaps) == the torch reference swap
    on float32 rows, int16 plane stacks and the float64 / int32 state columns, bitwise;
    odd widths take the scalar path, aligned ones the 16-byte one."""
    g = torch.Generator().manual_seed(3)
    K, R = 7, 40
    pairs = torch.tensor([3, 30, 0, 39, 12, 5, 21, 22], dtype=torch.int32)
    for cols in (2000, 333):
        HT = torch.randn((R * K, cols), generator=g)
        W = torch.randn((R * K, cols + 8), generator=g)[:, :cols]       # strided rows
        pl = torch.randint(-30000, 30000, (3, R * K, 64), generator=g, dtype=torch.int16)
        sf = torch.randn((3, R), generator=g, dtype=torch.float64)
        si = torch.randint(0, 100, (5, R), generator=g, dtype=torch.int32)
        ref = [t.clone() for t in (HT, W, pl, sf, si)]
        ops.rows_swap(pairs, K, ref[:3], ref[3], ref[4])
        dev = [t.cuda() for t in (HT, W, pl, sf, si)]
        ops.rows_swap(pairs.cuda(), K, dev[:3], dev[3], dev[4])
        for a, b in zip(ref, dev):
            assert torch.equal(a, b.cpu())
        # the reference really swapped: position 3 <-> 30
        assert torch.equal(ref[0][3 * K:4 * K], HT[30 * K:31 * K])
        assert torch.equal(ref[3][:, 30], sf[:, 3])


@pytest.mark.parametrize("K", [10, 20])
def test_swap_compaction_equals_gather_compaction(monkeypatch, K):
    """Single-K arena batches compact by in-place swaps of the movers only
    (_Batch._compact_swap): the run equals the gather-form compaction of the same layouts
    bit for bit (positions differ, per-replicate arithmetic does not)."""
    from cnmf_torch_amd.models import nmf
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(6000, 700, n_programs=10, seed=6)).cuda()
    seeds = list(range(40, 88))
    opts = nmf.NMFOptions(n_components=K, online_chunk_size=2000, online_chunk_max_iter=1000)
    monkeypatch.setenv("CNMF_COMPACT_FRAC_SMALL", "0.1")
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CNMF_COMPACT_SWAP", mode)
        out[mode] = nmf.NMFBatchSolver(X, opts).run(seeds)
    a, b = out["0"], out["1"]
    assert len(set(a.n_iter.tolist())) > 2
    np.testing.assert_array_equal(a.n_iter, b.n_iter)
    np.testing.assert_array_equal(a.err, b.err)
    assert torch.equal(a.W, b.W) and torch.equal(a.HT, b.HT)


@pytest.mark.parametrize("beta,K", [(1.0, 80), (0.0, 60), (1.5, 72), (0.5, 130)])
def test_beta_any_contract_matches_float64_reference(beta, K):
    """The rank-general beta contraction (KL beyond 64, IS / general beta beyond 56:
    library GEMMs + beta_any.hip's terms pass) == the float64 reference on both sides,
    with an inactive replicate (zero outputs) and the divergence sums."""
    from cnmf_torch_amd import ops
    from cnmf_torch_amd.ops import reference

    assert ops.beta_any_k(K, beta)
    g = torch.Generator().manual_seed(K)
    R, N, G = 3, 500, 301
    X = torch.rand((N, G), generator=g, dtype=torch.float64) * \
        (torch.rand((N, G), generator=g, dtype=torch.float64) < 0.4)
    HT = torch.rand((R, K, N), generator=g, dtype=torch.float64) / K
    W = torch.rand((R, K, G), generator=g, dtype=torch.float64)
    act = torch.tensor([1, 0, 1], dtype=torch.int32)
    d = dict(device="cuda", dtype=torch.float32)
    for side in ("h", "w"):
        s = {"h": 0, "w": 1}[side]
        nr, dr, lr = reference.beta_contract(s, X, HT, W, beta, 1e-16, True, s == 0, act)
        ng, dg, lg = ops.beta_contract(side, X.to(**d), HT.to(**d), W.to(**d), beta, 1e-16,
                                       want_loss=s == 0, active=act.cuda())
        for r in (0, 2):
            np.testing.assert_allclose(ng[r].cpu().double().numpy(), nr[r].numpy(), rtol=2e-4,
                                       atol=1e-6 * float(nr[r].abs().max()))
            if dr is not None:
                np.testing.assert_allclose(dg[r].cpu().double().numpy(), dr[r].numpy(),
                                           rtol=2e-4, atol=1e-6 * float(dr[r].abs().max()))
        assert float(ng[1].abs().max()) == 0.0
        assert (dg is None) == (dr is None)
        if s == 0:
            np.testing.assert_allclose(lg[[0, 2]].cpu().numpy(), lr[[0, 2]].numpy(), rtol=1e-4)
            assert float(lg[1]) == 0.0


@pytest.mark.parametrize("loss,K", [("kullback-leibler", 80), ("itakura-saito", 60)])
def test_beta_rank_beyond_panels_runs_native(loss, K, recwarn):
    """KL at K > 64 and IS at K > 56 factorise on the rank-general path (no eager routing,
    no warning) like the CPU engine of the same seeds."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    Xn = normalized_counts_matrix(600, 200, n_programs=6, seed=4)
    opts = NMFOptions(n_components=K, beta_loss=loss, online_chunk_size=300,
                      online_max_pass=3)
    g = NMFBatchSolver(torch.from_numpy(Xn).cuda(), opts).run([7, 8])
    c = NMFBatchSolver(torch.from_numpy(Xn), opts).run([7, 8])
    assert torch.isfinite(g.W).all() and (g.W >= 0).all()
    np.testing.assert_allclose(g.err, c.err, rtol=5e-3)
    assert not [w for w in recwarn.list if "eager" in str(w.message)]


def test_rank_general_batch_mode_and_pipeline_at_k_140(tmp_path, recwarn):
    """The rank-general solve under the batch-mode engine (fixed-step column splits) and
    through the cNMF pipeline (prepare -> factorize -> combine) at
    K = 140 on the GPU, no eager routing."""
    import pandas as pd

    from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix, simulate_counts

    Xn = normalized_counts_matrix(700, 260, n_programs=6, seed=5)
    opts = NMFOptions(n_components=140, mode="batch", batch_max_iter=30)
    g = NMFBatchSolver(torch.from_numpy(Xn).cuda(), opts).run([3, 4])
    c = NMFBatchSolver(torch.from_numpy(Xn), opts).run([3, 4])
    np.testing.assert_allclose(g.err, c.err, rtol=2e-3)
    X, cells, genes = simulate_counts(600, 300, 6, seed=2, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), fn)
    obj = cNMF(output_dir=str(tmp_path), name="k140")
    obj.prepare(fn, components=[140], n_iter=3, seed=1, num_highvar_genes=250, prewarm=False)
    obj.factorize(verbose=False)
    obj.combine()
    # (no consensus: at K = 140 on 250 genes some components die to exact zeros, whose
    # l2 normalisation is NaN -- in the reference's formula too, cnmf.py:1056)
    merged = load_df_from_npz(obj.paths["merged_spectra"] % 140)
    assert merged.shape == (3 * 140, 250) and np.isfinite(merged.values).all()
    assert not [w for w in recwarn.list if "eager" in str(w.message)]


def test_host_mapped_flags_match_copied_flags_bitwise(monkeypatch):
    """The fused passes' active flags stored by conv_update into alternating host-mapped
    slots (CNMF_HOST_FLAGS, default) give exactly the compactions -- and so the
    factorisations -- of the per-pass device->host copy, run after run."""
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.utils.synthetic import normalized_counts_matrix

    X = torch.from_numpy(normalized_counts_matrix(3000, 500, n_programs=8, seed=9)).cuda()
    opts = NMFOptions(n_components=8, online_chunk_size=1500)
    seeds = [[7 + 100 * i + j for j in range(24)] for i in range(3)]
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("CNMF_HOST_FLAGS", flag)
        solver = NMFBatchSolver(X, opts)
        out[flag] = [solver.run(s) for s in seeds]
    for a, b in zip(out["1"], out["0"]):
        assert torch.equal(a.W, b.W) and torch.equal(a.HT, b.HT)
        np.testing.assert_array_equal(a.err, b.err)
        np.testing.assert_array_equal(a.n_iter, b.n_iter)

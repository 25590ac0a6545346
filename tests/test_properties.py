"""Property-based tests (hypothesis) of the algorithmic contracts, SURVEY.md §4 items 1-2:
MU / HALS inner solves never increase their objective, batch Frobenius MU is monotone,
HALS reaches a KKT point, Philox draws are well-formed, and the cooperative / column-split
layouts of a solve change nothing but summation order."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
from cnmf_torch_amd.ops import reference
from cnmf_torch_amd.utils.rng import philox_matrix

SET = settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def _problem(seed, R, K, n):
    g = torch.Generator().manual_seed(seed)
    W = torch.rand((R, K, 3 * K + 5), generator=g, dtype=torch.float64) + 0.01
    gram = torch.bmm(W, W.transpose(1, 2))
    xt = torch.rand((R, K, n), generator=g, dtype=torch.float64)
    numer = torch.bmm(gram, xt) + 0.1 * torch.rand((R, K, n), generator=g, dtype=torch.float64)
    x0 = torch.rand((R, K, n), generator=g, dtype=torch.float64) + 0.05
    return x0, numer, gram


def _obj(x, numer, gram):
    # 0.5 x^T G x - numer . x per replicate (the NNLS objective up to a constant)
    return (0.5 * (x * torch.bmm(gram, x)).sum(dim=(1, 2)) - (numer * x).sum(dim=(1, 2)))


@SET
@given(seed=st.integers(0, 10_000), R=st.integers(1, 4), K=st.integers(1, 12),
       n=st.integers(1, 60), algo=st.sampled_from([0, 1]))
def test_inner_solve_objective_non_increasing(seed, R, K, n, algo):
    x, numer, gram = _problem(seed, R, K, n)
    prev = _obj(x, numer, gram)
    for _ in range(8):
        reference.solve(algo, x, numer, gram, None, 1, -1.0, 0.0, 0.0, 0.0, 1e-16, None, None,
                        None, 1, 0, 10)
        cur = _obj(x, numer, gram)
        assert torch.all(cur <= prev + 1e-9 * prev.abs().clamp(min=1.0)), (cur, prev)
        assert torch.all(x >= 0)
        prev = cur


@SET
@given(seed=st.integers(0, 10_000), K=st.integers(1, 8), n=st.integers(5, 40))
def test_hals_reaches_kkt_point(seed, K, n):
    x, numer, gram = _problem(seed, 1, K, n)
    reference.solve(1, x, numer, gram, None, 3000, 1e-13, 0.0, 0.0, 0.0, 1e-16, None, None, None,
                    1, 0, 10)
    grad = torch.bmm(gram, x) - numer                     # d/dx of the objective
    # KKT: grad >= 0 where x == 0, grad == 0 where x > 0 -> projected gradient vanishes
    pg = torch.where(x > 0, grad, torch.clamp(grad, max=0.0))
    scale = numer.abs().max().item() + 1.0
    assert pg.abs().max().item() < 1e-5 * scale


@settings(max_examples=8, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 1000), algo=st.sampled_from(["mu", "hals"]))
def test_batch_frobenius_error_monotone(seed, algo):
    rs = np.random.default_rng(seed)
    X = torch.from_numpy(rs.gamma(1.0, 1.0, (60, 25)) @ rs.gamma(1.0, 1.0, (25, 30)))
    errs = []
    for it in (1, 2, 4, 8, 16):
        opts = NMFOptions(n_components=4, mode="batch", algo=algo, batch_max_iter=it, tol=-1.0,
                          fp_precision="double", loss_every=1)
        errs.append(float(NMFBatchSolver(X, opts).run([seed + 1]).err[0]))
    assert all(b <= a * (1 + 1e-10) for a, b in zip(errs, errs[1:])), errs


@SET
@given(seed=st.integers(0, 2 ** 31 - 2), rows=st.integers(1, 50), cols=st.integers(1, 50),
       offset=st.integers(0, 1000))
def test_philox_uniform_open_interval_and_row_offset(seed, rows, cols, offset):
    u = philox_matrix(seed, 1, rows, cols, mode=1)
    assert u.shape == (rows, cols)
    assert np.all(u > 0) and np.all(u < 1)
    full = philox_matrix(seed, 1, rows + offset, cols, mode=1)
    np.testing.assert_array_equal(philox_matrix(seed, 1, rows, cols, mode=1, row_offset=offset),
                                  full[offset:])


@SET
@given(seed=st.integers(0, 10_000), R=st.integers(1, 3), K=st.integers(1, 6),
       n=st.integers(2, 80), nsplit=st.integers(2, 5))
def test_column_split_single_step_is_layout_invariant(seed, R, K, n, nsplit):
    """One fixed step split over column slices == unsplit (columns are independent)."""
    x, numer, gram = _problem(seed, R, K, n)
    a, b = x.clone(), x.clone()
    reference.solve(0, a, numer, gram, None, 1, -1.0, 0.0, 0.0, 0.0, 1e-16, None, None, None,
                    1, 0, 10)
    reference.solve(0, b, numer, gram, None, 1, -1.0, 0.0, 0.0, 0.0, 1e-16, None, None, None,
                    nsplit, 0, 10)
    torch.testing.assert_close(a, b, rtol=0, atol=0)

"""Fused residual -> restriction (`KronTransfer.resid_restrict`, `poms_resid_restrict`)
against the oracle's ``R (b - A x)`` (`sources/mg_jac.py:93-94`: ``rf = bf - Af.dot(xf)``,
``rc = R.dot(rf)``) and against the unfused device pair (residual, then restriction).

The fused pass sums ``R b - (R A) x`` in another order than ``R (b - A x)``, so the
comparison is normwise relative: 1e-13 on random x (no cancellation), and 1e-13 of
``|R b| + |R A x|`` where x nearly solves ``A x = b`` (the residual is then small
against both terms, the same cancellation the reference's own subtraction has).
"""
import numpy as np
import pytest
import torch

from poms_amd.splines import assemble_1d, uniform_knots

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _kron_restrict(P, v, nd):
    if nd == 3:
        return np.einsum("ia,jb,kc,ijk->abc", P, P, P, v).reshape(-1)
    if nd == 2:
        return (P.T @ v @ P).reshape(-1)
    return P.T @ v


def _setup(nd, p, Nf, Nc, form, align=True):
    from poms_amd.mg import two_level_setup_1d
    from poms_amd.multilevels import KronTransfer
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    _, _, P1 = two_level_setup_1d(p, uniform_knots(p, Nf), uniform_knots(p, Nc))
    M, K = assemble_1d(uniform_knots(p, Nf), p)
    n = Nf + p
    V = StencilVectorSpace([n] * nd, [p] * nd, align=align)
    if form == "sum":
        A = KronOperator.laplace(V, [M] * nd, [K] * nd, mass_coef=0.75)
    else:
        rng = np.random.default_rng(5)
        A = KronOperator.product(V, [M + 0.1 * rng.standard_normal(M.shape) * (M != 0) for _ in range(nd)])
    return V, A, KronTransfer(V, [P1] * nd), P1, n


CASES = [(3, 3, 32, 8, "sum"), (3, 2, 24, 4, "sum"), (3, 1, 16, 4, "single"), (3, 5, 20, 4, "sum"),
         (3, 3, 40, 20, "sum"), (2, 3, 64, 8, "sum"), (2, 2, 48, 16, "single"), (2, 4, 192, 12, "sum"),
         (1, 3, 64, 8, "sum"), (1, 2, 40, 4, "single")]


@pytest.mark.parametrize("nd,p,Nf,Nc,form", CASES)
def test_resid_restrict_random(gpu, nd, p, Nf, Nc, form):
    V, A, tr, P1, n = _setup(nd, p, Nf, Nc, form)
    assert tr.set_operator(A)
    rng = np.random.default_rng(11)
    xg, bg = rng.uniform(-1, 1, (n,) * nd), rng.uniform(-1, 1, (n,) * nd)
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    rc = tr.resid_restrict(A, b, x).cpu().numpy()
    Ax = (A.tosparse() @ xg.reshape(-1)).reshape(xg.shape)
    want = _kron_restrict(P1, bg - Ax, nd)
    assert rel(rc, want) <= 1e-13
    # the unfused device pair
    r = A.residual(b, x)
    rc2 = tr.restrict(r).cpu().numpy()
    assert rel(rc, rc2) <= 1e-13


@pytest.mark.parametrize("nd,p,Nf,Nc", [(3, 3, 32, 8), (2, 3, 64, 8)])
def test_resid_restrict_small_residual(gpu, nd, p, Nf, Nc):
    """x nearly solves A x = b: the fused error is bounded by rounding of |R b| + |R A x|."""
    V, A, tr, P1, n = _setup(nd, p, Nf, Nc, "sum")
    S = A.tosparse().tocsr()
    f = 1 + 0.5 * np.sin(np.pi * np.linspace(0, 1, n))    # smooth x (R A x does not cancel)
    xg = f
    for _ in range(nd - 1):
        xg = np.multiply.outer(xg, f)
    bg = (S @ xg.reshape(-1)).reshape(xg.shape)           # x solves A x = b ...
    xg = xg * (1 + 1e-8)                                  # ... up to a 1e-8 perturbation
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    rc = tr.resid_restrict(A, b, x).cpu().numpy()
    Ax = (S @ xg.reshape(-1)).reshape(xg.shape)
    want = _kron_restrict(P1, bg - Ax, nd)
    scale = np.linalg.norm(_kron_restrict(P1, np.abs(bg), nd)) + np.linalg.norm(_kron_restrict(P1, np.abs(Ax), nd))
    assert np.linalg.norm(rc - want) <= 1e-13 * scale
    assert np.linalg.norm(want) > 1e-10 * scale   # (not vacuous: R r is 1e3 x the rounding bound)


def test_resid_restrict_ignores_ghosts(gpu):
    """x's ghost regions are not read: garbage there leaves the result unchanged."""
    V, A, tr, P1, n = _setup(3, 3, 24, 8, "sum")
    rng = np.random.default_rng(4)
    xg, bg = rng.uniform(-1, 1, (n,) * 3), rng.uniform(-1, 1, (n,) * 3)
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    rc = tr.resid_restrict(A, b, x).clone()
    own = V.interior(x._data).clone()
    x._data.fill_(1e30)
    V.interior(x._data).copy_(own)
    assert torch.equal(tr.resid_restrict(A, b, x), rc)


def test_resid_restrict_refuses_banded(gpu):
    """Coarse extents > 32 (banded transfers): set_operator says no, and the multilevel
    V-cycle keeps residual + restriction on those levels."""
    V, A, tr, P1, n = _setup(2, 3, 128, 64, "sum")
    assert not tr.set_operator(A)
    with pytest.raises(ValueError):
        tr.resid_restrict(A, V.zeros(), V.zeros())


@pytest.mark.parametrize("nd,p,N", [(3, 3, 32), (2, 3, 64), (3, 2, 16)])
def test_vcycle_fused_matches_unfused(gpu, nd, p, N):
    """The two-level V-cycle with the fused residual -> restriction equals the
    reference's order (residual vector, then restriction) to 1e-10, same niter."""
    from poms_amd.mg import TwoLevelVCycle
    mgf = TwoLevelVCycle(p, N, 8 if N >= 32 else 4, ndim=nd, tol=0.0, maxiter=4, fused_restrict=True)
    mgu = TwoLevelVCycle(p, N, 8 if N >= 32 else 4, ndim=nd, tol=0.0, maxiter=4, fused_restrict=False)
    assert mgf.fused_restrict and not mgu.fused_restrict
    xf, ipf, iqf = mgf.cycle(mgf.rhs_ones())
    xu, ipu, iqu = mgu.cycle(mgu.rhs_ones())
    assert ipf["niter"] == ipu["niter"] and iqf["niter"] == iqu["niter"]
    assert rel(xf.toarray(), xu.toarray()) <= 1e-10

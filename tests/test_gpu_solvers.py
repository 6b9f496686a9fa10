"""GPU parity of pcg / damped_jacobi / jacobi / two-level V-cycle vs the oracle.

Tolerance after m PCG iterations or a V-cycle: <= 1e-9 normwise relative AND
identical ``niter``; fixed-count comparisons use ``tol=0``.
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, uniform_knots

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def parity_bound(run_oracle, ndim, n, M, K):
    """Tolerance for an iterate comparison: 1e-9, or -- where the reference's own
    algorithm amplifies roundoff (damped Jacobi with omega = 2/3 is divergent on
    the high-frequency modes once lambda_max(D^-1 A) > 3, e.g. 3D p = 3) -- 20x
    the disagreement between two CPU restatements of the reference that differ
    only in summation order (sparse CSR vs term-by-term Kronecker apply)."""
    Acsr = orc.kron_sum_csr(M, K)
    a1 = lambda v: Acsr @ v
    a2 = lambda v: orc.kron_sum_apply(v.reshape((n,) * ndim), M, K).reshape(-1)
    x1, x2 = run_oracle(a1), run_oracle(a2)
    return max(1e-9, 20.0 * rel(x2, x1)), x1


def _problem(ndim, N, p):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    Ms, Ks = [M] * ndim, [K] * ndim
    Acsr = orc.kron_sum_csr(Ms, Ks)
    D = orc.kron_sum_diag(Ms, Ks).reshape(-1)
    return V, A, Acsr, D, n


@pytest.mark.parametrize("ndim,N,p", [(2, 16, 1), (2, 12, 3), (3, 8, 2), (3, 10, 3)])
@pytest.mark.parametrize("maxiter", [1, 4, 10])
def test_damped_jacobi(gpu, ndim, N, p, maxiter):
    from poms_amd.solvers import damped_jacobi
    V, A, Acsr, D, n = _problem(ndim, N, p)
    x0 = np.fromfunction(lambda *i: sum(i) + 1.0, (n,) * ndim)
    b = (Acsr @ x0.reshape(-1)).reshape(x0.shape)
    bv = V.zeros().from_numpy(b)
    for tol in (0.0, 1e-6):
        x = damped_jacobi(A, bv, tol=tol, maxiter=maxiter).to_local_numpy()
        xr = orc.damped_jacobi(lambda v: Acsr @ v, D, b.reshape(-1), tol=tol, maxiter=maxiter)
        assert rel(x.reshape(-1), xr) <= 1e-12
    # with a starting guess
    xs = np.random.default_rng(0).uniform(-1, 1, b.shape)
    x = damped_jacobi(A, bv, x0=V.zeros().from_numpy(xs), tol=0.0, maxiter=maxiter).to_local_numpy()
    xr = orc.damped_jacobi(lambda v: Acsr @ v, D, b.reshape(-1), x0=xs.reshape(-1), tol=0.0, maxiter=maxiter)
    assert rel(x.reshape(-1), xr) <= 1e-12


@pytest.mark.parametrize("ndim,N,p", [(2, 16, 1), (2, 12, 3), (3, 10, 3)])
def test_pcg_fixed_count(gpu, ndim, N, p):
    from poms_amd.solvers import damped_jacobi, pcg
    V, A, Acsr, D, n = _problem(ndim, N, p)
    b = np.ones((n,) * ndim)
    bv = V.zeros().from_numpy(b)
    apply = lambda v: Acsr @ v
    Ms, Ks = [A.M[0]] * ndim, [A.K[0]] * ndim
    for m in (1, 2, 3, 6):
        x, info = pcg(A, lambda AA, r: damped_jacobi(AA, r, tol=0.0), bv, tol=0.0, maxiter=m)
        run = lambda ap: orc.pcg(ap, lambda r: orc.damped_jacobi(ap, D, r, tol=0.0), b.reshape(-1),
                                 tol=0.0, maxiter=m)[0]
        tol, xr = parity_bound(run, ndim, n, Ms, Ks)
        if m <= 3:   # <= 1e-9 after m iterations -- no roundoff-spread allowance
            tol = 1e-9
        ir = orc.pcg(apply, lambda r: orc.damped_jacobi(apply, D, r, tol=0.0), b.reshape(-1), tol=0.0, maxiter=m)[1]
        assert info["niter"] == ir["niter"] == m
        assert rel(x.to_local_numpy().reshape(-1), xr) <= tol
        if tol == 1e-9:
            assert info["res_norm"] == pytest.approx(ir["res_norm"], rel=1e-8)


@pytest.mark.parametrize("ndim,N,p", [(2, 16, 1), (3, 8, 3)])
def test_pcg_reference_defaults(gpu, ndim, N, p):
    """The V-cycle's call: pcg(A, damped_jacobi, b, tol=1e-6, maxiter=10) (`sources/mg_jac.py:87`)."""
    from poms_amd.solvers import damped_jacobi, pcg
    V, A, Acsr, D, n = _problem(ndim, N, p)
    x0 = np.fromfunction(lambda *i: sum(i) + 1.0, (n,) * ndim)
    b = (Acsr @ x0.reshape(-1)).reshape(x0.shape)
    apply = lambda v: Acsr @ v
    x, info = pcg(A, damped_jacobi, V.zeros().from_numpy(b), tol=1e-6, maxiter=10)
    xr, ir = orc.pcg(apply, lambda r: orc.damped_jacobi(apply, D, r), b.reshape(-1), tol=1e-6, maxiter=10)
    run = lambda ap: orc.pcg(ap, lambda r: orc.damped_jacobi(ap, D, r), b.reshape(-1), tol=1e-6, maxiter=10)[0]
    tol, _ = parity_bound(run, ndim, n, [A.M[0]] * ndim, [A.K[0]] * ndim)
    assert info["niter"] == ir["niter"]
    assert info["success"] == ir["success"]
    assert rel(x.to_local_numpy().reshape(-1), xr) <= tol


def test_jacobi_point(gpu):
    from poms_amd.solvers import jacobi
    V, A, Acsr, D, n = _problem(2, 9, 2)
    b = np.random.default_rng(4).uniform(-1, 1, (n, n))
    x = jacobi(A, V.zeros().from_numpy(b)).to_local_numpy()
    assert rel(x.reshape(-1), orc.jacobi(D, b.reshape(-1))) <= 1e-15


@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("ndim,p,Nf,Nc", [(2, 1, 16, 8), (2, 3, 32, 8), (3, 2, 16, 8), (3, 3, 16, 4)])
def test_two_level_vcycle(gpu, ndim, p, Nf, Nc, align):
    from poms_amd.mg import TwoLevelVCycle
    mg = TwoLevelVCycle(p, Nf, Nc, ndim=ndim, align=align)
    assert mg.space.aligned == align
    b = mg.rhs_ones()
    x, ipre, ipos = mg.cycle(b)
    Ms, Ks = [mg.M1d] * ndim, [mg.K1d] * ndim
    xr, rpre, rpos = orc.vcycle_two_level(Ms, Ks, mg.P1, np.ones((mg.n,) * ndim))
    xr2, _, _ = orc.vcycle_two_level(Ms, Ks, mg.P1, np.ones((mg.n,) * ndim), reorder=True)
    tol = max(1e-9, 20.0 * rel(xr2, xr))
    assert ipre["niter"] == rpre["niter"] and ipos["niter"] == rpos["niter"]
    assert rel(x.to_local_numpy(), xr) <= tol


@pytest.mark.parametrize("ndim,p,Nf,Nc", [(2, 1, 16, 8), (2, 3, 32, 8), (3, 2, 16, 8), (3, 3, 24, 8)])
def test_two_level_vcycle_glt_post(gpu, ndim, p, Nf, Nc):
    """`sources/mg_glt.py`: pre pcg + damped Jacobi, coarse correction, GLT
    post-smoother pcg_glt(maxiter = p + 1) with the collocation Kron solve."""
    from poms_amd.mg import TwoLevelVCycle
    from poms_amd.splines import collocation_cardinal_splines, dense_to_band, band_to_dense
    mg = TwoLevelVCycle(p, Nf, Nc, ndim=ndim, post_smoother="glt")
    b = mg.rhs_ones()
    x, ipre, ipos = mg.cycle(b)
    Cd = band_to_dense(dense_to_band(collocation_cardinal_splines(p, mg.n), p))
    Ms, Ks = [mg.M1d] * ndim, [mg.K1d] * ndim
    ones = np.ones((mg.n,) * ndim)
    xr, rpre, rpos = orc.vcycle_two_level(Ms, Ks, mg.P1, ones, glt=[Cd] * ndim)
    xr2, _, _ = orc.vcycle_two_level(Ms, Ks, mg.P1, ones, glt=[Cd] * ndim, reorder=True)
    tol = max(1e-9, 20.0 * rel(xr2, xr))
    assert ipre["niter"] == rpre["niter"] and ipos["niter"] == rpos["niter"] <= p + 1
    assert rel(x.to_local_numpy(), xr) <= tol

def test_transfer_restrict_prolong(gpu):
    from poms_amd.mg import TwoLevelVCycle
    import torch
    mg = TwoLevelVCycle(3, 32, 8, ndim=3)
    rng = np.random.default_rng(9)
    f = rng.uniform(-1, 1, (mg.n,) * 3)
    fv = mg.space.zeros().from_numpy(f)
    rc = mg.transfer.restrict(fv).cpu().numpy()
    P = mg.P1
    ref = np.einsum("ia,jb,kc,ijk->abc", P, P, P, f).reshape(-1)
    assert rel(rc, ref) <= 1e-13
    xc = rng.uniform(-1, 1, rc.shape)
    out = mg.space.zeros().from_numpy(f)
    mg.transfer.prolong_add(torch.from_numpy(xc).cuda(), out)
    ref2 = f + np.einsum("ia,jb,kc,abc->ijk", P, P, P, xc.reshape((P.shape[1],) * 3))
    assert rel(out.to_local_numpy(), ref2) <= 1e-13


@pytest.mark.parametrize("ndim,p,Nf,Nc,maxiters", [(2, 1, 32, 4, None), (2, 3, 32, 8, [4, 6]),
                                                   (3, 2, 16, 4, [3, 10])])
def test_multilevel_vcycle(gpu, ndim, p, Nf, Nc, maxiters):
    """MultilevelVCycle against the oracle's recursive cycle with
    materialised Galerkin operators R A P on every level: same iteration counts,
    iterates within the parity bound."""
    from poms_amd.mg import MultilevelVCycle
    mg = MultilevelVCycle(p, Nf, Nc, ndim=ndim, maxiters=maxiters)
    assert mg.nlevels >= 3
    b = mg.rhs_ones()
    x, infos = mg.cycle(b)
    ones = np.ones((mg.spaces[0].npts[0],) * ndim)
    Ms, Ks = [[mg.M1d[0]] * ndim], [[mg.K1d[0]] * ndim]
    xr, rinfos = orc.vcycle_multilevel(Ms, Ks, mg.P1, ones, maxiters=mg.maxiters)
    xr2, _ = orc.vcycle_multilevel(Ms, Ks, mg.P1, ones, maxiters=mg.maxiters, reorder=True)
    tol = max(1e-9, 20.0 * rel(xr2, xr))
    for l in range(mg.nlevels - 1):
        assert infos[l][0]["niter"] == rinfos[l][0]["niter"] and infos[l][1]["niter"] == rinfos[l][1]["niter"], l
    assert rel(x.to_local_numpy(), xr) <= tol


def test_multilevel_converges_h_independently(gpu):
    """Repeated multilevel cycles solve -Δu+u = 1 (2D, p = 2) with a contraction per
    cycle that does not degrade as the grid is refined (the O(n) claim of
    `slides/content.tex:42` that motivates SURVEY §8f rank 1)."""
    from poms_amd.mg import MultilevelVCycle
    rates = []
    for N in (32, 128):
        mg = MultilevelVCycle(2, N, 4, ndim=2)
        mg.maxiters = [2] * (mg.nlevels - 1)
        b = mg.rhs_ones()
        x = None
        res = []
        for _ in range(4):
            x, _ = mg.cycle(b, x0=x)
            r = mg.A.residual(b, x)
            res.append(np.sqrt(r.dot(r)))
        rates.append((res[-1] / res[0]) ** (1.0 / 3))
        assert res[-1] < 1e-3 * res[0]
    assert rates[1] <= 2.0 * rates[0] + 0.05


@pytest.mark.parametrize("ndim,p,Nf", [(2, 3, 80), (3, 2, 72)])
def test_transfer_banded(gpu, ndim, p, Nf):
    """Restriction / prolongation with coarse extents > 32 (the banded gather kernels
    of the multilevel hierarchy) against dense einsum."""
    import torch
    from poms_amd.mg import two_level_setup_1d
    from poms_amd.multilevels import KronTransfer
    from poms_amd.splines import uniform_knots
    from poms_amd.stencil import StencilVectorSpace
    _, _, P1 = two_level_setup_1d(p, uniform_knots(p, Nf), uniform_knots(p, Nf // 2))
    n = P1.shape[0]
    assert P1.shape[1] > 32
    V = StencilVectorSpace([n] * ndim, [p] * ndim, align=True)
    tr = KronTransfer(V, [P1] * ndim)
    rng = np.random.default_rng(4)
    f = rng.uniform(-1, 1, (n,) * ndim)
    rc = tr.restrict(V.zeros().from_numpy(f)).cpu().numpy()
    sub = "ia,jb,kc,ijk->abc" if ndim == 3 else "ia,jb,ij->ab"
    ref = np.einsum(sub, *([P1] * ndim), f, optimize=True).reshape(-1)
    assert rel(rc, ref) <= 1e-13
    xc = rng.uniform(-1, 1, rc.shape)
    out = V.zeros().from_numpy(f)
    tr.prolong_add(torch.from_numpy(xc).cuda(), out)
    sub2 = "ia,jb,kc,abc->ijk" if ndim == 3 else "ia,jb,ab->ij"
    ref2 = f + np.einsum(sub2, *([P1] * ndim), xc.reshape((P1.shape[1],) * ndim), optimize=True)
    assert rel(out.to_local_numpy(), ref2) <= 1e-13


@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("maxiter", [1, 2, 3])
def test_two_level_vcycle_fixed_count_3d_p3(gpu, maxiter, align):
    """The headline order (3D p = 3) pinned at the SURVEY §8c floor: the reference's
    V-cycle schedule (`sources/mg_jac.py:84-119`, tol = 1e-6) with pre/post
    pcg(maxiter <= 3), where the roundoff amplification of omega = 2/3 Jacobi is
    still negligible (two oracle orderings agree to ~5e-16): <= 1e-9 and identical
    niter, no spread allowance."""
    from poms_amd.mg import TwoLevelVCycle
    mg = TwoLevelVCycle(3, 16, 4, ndim=3, maxiter=maxiter, align=align)
    x, ipre, ipos = mg.cycle(mg.rhs_ones())
    xr, rpre, rpos = orc.vcycle_two_level([mg.M1d] * 3, [mg.K1d] * 3, mg.P1, np.ones((mg.n,) * 3), maxiter=maxiter)
    assert ipre["niter"] == rpre["niter"] == maxiter and ipos["niter"] == rpos["niter"] == maxiter
    assert ipre["success"] == rpre["success"] and ipos["success"] == rpos["success"]
    assert rel(x.to_local_numpy(), xr) <= 1e-9


@pytest.mark.parametrize("maxiter", [3, 10])
def test_two_level_vcycle_reference_coarse_convention_3d(gpu, maxiter):
    """3D p = 3 on the reference driver's knots: ``nc = 8`` BASIS FUNCTIONS on the coarse
    grid (`sources/mg_jac.py:25,28`: ``make_open_knots(p, nc)``, 5 cells at p = 3) and a
    fine grid of ``nf = 19`` basis functions, whose union with the inserted knots is
    non-uniform (23 fine DOF per axis).  maxiter = 3 at 1e-9; the reference's
    maxiter = 10 with identical niter and the roundoff-spread bound."""
    from poms_amd.mg import TwoLevelVCycle
    from poms_amd.splines import make_open_knots
    Tf, Tc = make_open_knots(3, 19), make_open_knots(3, 8)
    mg = TwoLevelVCycle(3, 0, 0, ndim=3, knots_fine=Tf, knots_coarse=Tc, maxiter=maxiter)
    assert mg.P1.shape == (23, 8)
    x, ipre, ipos = mg.cycle(mg.rhs_ones())
    ones = np.ones((mg.n,) * 3)
    xr, rpre, rpos = orc.vcycle_two_level([mg.M1d] * 3, [mg.K1d] * 3, mg.P1, ones, maxiter=maxiter)
    tol = 1e-9
    if maxiter > 3:
        xr2, _, _ = orc.vcycle_two_level([mg.M1d] * 3, [mg.K1d] * 3, mg.P1, ones, maxiter=maxiter, reorder=True)
        tol = max(1e-9, 20.0 * rel(xr2, xr))
    assert ipre["niter"] == rpre["niter"] and ipos["niter"] == rpos["niter"]
    assert rel(x.to_local_numpy(), xr) <= tol


@pytest.mark.parametrize("convention", ["cells", "mg_jac"])
def test_two_level_vcycle_1d_p2_n128(gpu, convention):
    """BASELINE config 1: 1D Poisson p = 2, 128 cells, Jacobi-smoothed two-level
    V-cycle with the reference schedule (pcg(tol=1e-6, maxiter=10) pre/post).
    ``cells``: 8 coarse cells nested in 128 (130 fine DOF); ``mg_jac``: the
    reference's ``make_open_knots(p, 8)`` coarse / ``make_open_knots(p, 130)`` fine
    knots (`sources/mg_jac.py:25-35`).  Runs the 1D operator, smoother and the
    ``KronTransfer`` 1D embedding on the device."""
    from poms_amd.mg import TwoLevelVCycle
    from poms_amd.splines import make_open_knots
    if convention == "cells":
        mg = TwoLevelVCycle(2, 128, 8, ndim=1)
        assert mg.n == 130
    else:
        mg = TwoLevelVCycle(2, 0, 0, ndim=1, knots_fine=make_open_knots(2, 130), knots_coarse=make_open_knots(2, 8))
    x, ipre, ipos = mg.cycle(mg.rhs_ones())
    ones = np.ones(mg.n)
    xr, rpre, rpos = orc.vcycle_two_level([mg.M1d], [mg.K1d], mg.P1, ones)
    xr2, _, _ = orc.vcycle_two_level([mg.M1d], [mg.K1d], mg.P1, ones, reorder=True)
    assert ipre["niter"] == rpre["niter"] and ipos["niter"] == rpos["niter"]
    assert ipre["success"] == rpre["success"] and ipos["success"] == rpos["success"]
    assert rel(x.to_local_numpy(), xr) <= max(1e-9, 20.0 * rel(xr2, xr))
    # repeated cycles converge to the direct solution of A u = 1
    from oracle.poms_oracle import kron_sum_csr
    from scipy.sparse.linalg import spsolve
    u = spsolve(kron_sum_csr([mg.M1d], [mg.K1d]).tocsc(), ones)
    xk = x
    for _ in range(3):
        xk, _, _ = mg.cycle(mg.rhs_ones(), x0=xk)
    assert rel(xk.to_local_numpy(), u) <= 1e-8


@pytest.mark.parametrize("ndim,N,p", [(2, 12, 3), (3, 8, 2)])
def test_damped_jacobi_maxiter2_stops_after_sweep1(gpu, ndim, N, p):
    """maxiter = 2 from x0 = None with ||dr_1||^2 < tol^2: the reference stops after
    sweep 1 and returns x1 (`sources/solvers.py:219-222`).  Covers the lazily read
    two-sweeps-from-zero path, whose loop never runs at maxiter = 2."""
    from poms_amd.solvers import damped_jacobi
    V, A, Acsr, D, n = _problem(ndim, N, p)
    b = np.random.default_rng(3).uniform(0.5, 1.0, (n,) * ndim)
    tol = 1e-6
    dr1 = (2.0 / 3.0) * b.reshape(-1) / D
    for frac in (0.5, 2.0):   # ||dr_1||^2 = frac * tol^2: stop after sweep 1, or run both
        bs = b * np.sqrt(frac) * tol / np.linalg.norm(dr1)
        x = damped_jacobi(A, V.zeros().from_numpy(bs), tol=tol, maxiter=2).to_local_numpy()
        xr = orc.damped_jacobi(lambda v: Acsr @ v, D, bs.reshape(-1), tol=tol, maxiter=2)
        assert rel(x.reshape(-1), xr) <= 1e-12, frac
        if frac < 1:
            assert rel(x.reshape(-1), (2.0 / 3.0) * bs.reshape(-1) / D) <= 1e-14


@pytest.mark.parametrize("ndim,N,p,scale,x0,tol,maxiter", [
    (3, 20, 3, 1.0, False, 1e-6, 10),      # from-zero sweeps (3D), all iterations
    (3, 20, 3, 1.0, True, 1e-6, 10),
    (2, 64, 3, 1.0, False, 1e-6, 10),      # diagonal scaling first (2D)
    (3, 16, 2, 1e-5, False, 1e-6, 10),     # damped Jacobi stops after a few sweeps
    (3, 16, 3, 1e-9, False, 1e-6, 10),     # ... after sweep 1 (x1 re-formed)
    (2, 40, 1, 1e-9, True, 1e-6, 10),
    (3, 16, 3, 1.0, False, 0.5, 10),       # pcg stops early
    (3, 12, 2, 1.0, True, 1e-6, 1),
    (2, 24, 2, 1.0, False, 1e-6, 0),
    # large grids: a damped-Jacobi early stop abandons a queued sweep that is still
    # running when the next psolve re-arms host slots (advisor finding, round 2)
    (3, 128, 2, 1e-8, False, 1e-6, 4),
    (3, 128, 3, 1e-10, False, 1e-6, 3),
    (3, 96, 3, 1e-7, True, 1e-6, 4),
    # 2D p = 3 with the lookahead: two sweeps per launch; damped Jacobi stopping at
    # various sweeps, inside a two-sweep launch (x_k re-formed) or after it
    (2, 64, 3, 1e-4, False, 1e-6, 10),
    (2, 64, 3, 1e-6, False, 1e-6, 10),
    (2, 64, 3, 1e-7, True, 1e-6, 10),
    (2, 150, 3, 3e-8, False, 1e-6, 10),
    (2, 150, 3, 1e-9, True, 1e-6, 10),
])
@pytest.mark.parametrize("lookahead", ["0", "1"])
def test_native_pcg_matches_python_loop(gpu, monkeypatch, lookahead, ndim, N, p, scale, x0, tol, maxiter):
    """poms_pcg_jacobi (the whole pcg + damped-Jacobi loop in C) == the Python device
    loop, bitwise: same launches, same device scalars, same stop decisions -- with the
    stop tests read one sweep late, and two sweeps late over a fourth buffer
    (POMS_PCG_LOOKAHEAD=1: up to two abandoned sweeps past an early stop)."""
    monkeypatch.setenv("POMS_PCG_LOOKAHEAD", lookahead)
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    rng = np.random.default_rng(N + p)
    b = V.zeros().from_numpy(scale * rng.standard_normal((n,) * ndim))
    xi = V.zeros().from_numpy(rng.standard_normal((n,) * ndim)) if x0 else None
    assert solvers._native_ok(A, V)
    out = {}
    for native in ("0", "1"):
        monkeypatch.setenv("POMS_NATIVE_PCG", native)
        x, info = solvers.pcg(A, solvers.damped_jacobi, b, x0=xi, tol=tol, maxiter=maxiter)
        out[native] = (x.to_local_numpy(), info)
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    assert out["1"][1]["niter"] == out["0"][1]["niter"]
    assert out["1"][1]["success"] == out["0"][1]["success"]
    assert out["1"][1]["res_norm"] == out["0"][1]["res_norm"]


@pytest.mark.parametrize("ndim,N,p,scale,x0,tol,maxiter", [
    (2, 64, 3, 1.0, False, 1e-6, 10),      # the 2D default (lookahead on)
    (3, 20, 3, 1.0, True, 1e-6, 10),       # v5 on aligned tiles
    (3, 16, 2, 1e-5, False, 1e-6, 10),     # damped Jacobi stops early
    (2, 40, 1, 1e-9, True, 1e-6, 10),
])
@pytest.mark.parametrize("lookahead", ["0", "1"])
def test_native_pcg_matches_python_loop_aligned_layout(gpu, monkeypatch, lookahead, ndim, N, p, scale, x0, tol,
                                                       maxiter):
    """The same bitwise check on the V-cycle's line-aligned layout (align=True: the
    work vectors start `shift` doubles into their buffers).  The lookahead's fourth
    buffer takes their 128-B phase, so the flat vector kernels and v5's aligned
    tiles run on it as on the others (advisor, round 4: a raw hipMalloc sent its
    updates to the per-row fall-back and v5 to its unaligned tiles)."""
    monkeypatch.setenv("POMS_PCG_LOOKAHEAD", lookahead)
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim, align=True)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    rng = np.random.default_rng(N + p + 1)
    b = V.zeros().from_numpy(scale * rng.standard_normal((n,) * ndim))
    xi = V.zeros().from_numpy(rng.standard_normal((n,) * ndim)) if x0 else None
    assert solvers._native_ok(A, V)
    out = {}
    for native in ("0", "1"):
        monkeypatch.setenv("POMS_NATIVE_PCG", native)
        x, info = solvers.pcg(A, solvers.damped_jacobi, b, x0=xi, tol=tol, maxiter=maxiter)
        out[native] = (x.to_local_numpy(), info)
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    for k in ("niter", "success", "res_norm"):
        assert out["1"][1][k] == out["0"][1][k], k


@pytest.mark.parametrize("cap", ["0", "16"])
@pytest.mark.parametrize("ndim,N,p,scale", [(3, 20, 3, 1.0), (2, 64, 3, 1.0), (3, 16, 2, 1e-5)])
def test_native_pcg_device_reduction_fallback(gpu, monkeypatch, cap, ndim, N, p, scale):
    """The single-rank native loop's device-reduction fall-back (advisor, round 3):
    POMS_HOST_PARTIALS=0 reduces every host-read norm on the device; a cap of 16
    blocks takes the too-many-blocks branch for launches wider than that.  Both must
    equal the Python device loop bitwise, like the host-partials default."""
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    b = V.zeros().from_numpy(scale * np.random.default_rng(N).standard_normal((n,) * ndim))
    out = {}
    for native in ("0", "1"):
        monkeypatch.setenv("POMS_NATIVE_PCG", native)
        monkeypatch.setenv("POMS_HOST_PARTIALS", cap)
        x, info = solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=10)
        out[native] = (x.to_local_numpy(), info)
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    for k in ("niter", "success", "res_norm"):
        assert out["1"][1][k] == out["0"][1][k], k


@pytest.mark.parametrize("ndim,N,p,scale,x0,tol,maxiter", [
    (2, 64, 3, 1.0, False, 1e-6, 10),      # no stop test fires: the speculative run stands
    (2, 64, 3, 1.0, True, 1e-6, 10),       # (with x0)
    (3, 20, 3, 1.0, True, 1e-6, 4),        # 3D: sweeps 1-2 from zero in one launch
    (3, 16, 2, 1e-5, False, 1e-6, 10),     # damped Jacobi stops: repeated step by step
    (2, 40, 1, 1e-9, True, 1e-6, 10),      # ... with x0 restored first
    (3, 16, 3, 1.0, False, 0.5, 10),       # pcg stops early
])
def test_speculative_pcg_matches_step_by_step(gpu, monkeypatch, ndim, N, p, scale, x0, tol, maxiter):
    """poms_pcg_jacobi's speculative mode (every launch of the smoother call queued, the
    stop tests evaluated once the stream drains; POMS_PCG_SPEC=1) == the step-by-step
    loop (POMS_PCG_SPEC=0) == the Python device loop, bitwise -- including the cases
    where a stop test fires and the call is repeated from the restored x0."""
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    rng = np.random.default_rng(N + 7 * p)
    b = V.zeros().from_numpy(scale * rng.standard_normal((n,) * ndim))
    xi = V.zeros().from_numpy(rng.standard_normal((n,) * ndim)) if x0 else None
    out = {}
    xin = None if xi is None else xi.copy()   # one buffer for every native call: the graph key repeats
    for mode in ("python", "0", "1", "g", "g2"):
        monkeypatch.setenv("POMS_NATIVE_PCG", "0" if mode == "python" else "1")
        monkeypatch.setenv("POMS_PCG_SPEC", {"python": "0", "0": "0"}.get(mode, "1"))
        monkeypatch.setenv("POMS_PCG_GRAPH", "1" if mode.startswith("g") else "0")
        if xi is not None:
            xin._data.copy_(xi._data)
        x, info = solvers.pcg(A, solvers.damped_jacobi, b, x0=xin, tol=tol, maxiter=maxiter,
                              _x0_owned=mode != "python")
        out[mode] = (x.to_local_numpy(), info)
        del x
    st = A.spec_stats
    caps, hits = st["captures"], st["replays"]
    assert st["calls"] == 3
    if x0:   # same b, x, work and options: "g" captured, "g2" replayed
        assert caps == 1 and hits == 1, (caps, hits)
    else:    # (x = V.zeros() per call: the allocator decides whether the key repeats)
        assert caps + hits == 2, (caps, hits)
    for mode in ("0", "1", "g", "g2"):
        np.testing.assert_array_equal(out[mode][0], out["python"][0])
        for k in ("niter", "success", "res_norm"):
            assert out[mode][1][k] == out["python"][1][k], (mode, k)


def test_graph_replay_records_launch_timing(gpu, monkeypatch):
    """Speculative calls replayed from a captured graph: the timed launches are event
    nodes of the graph, recorded again by every replay."""
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, 16
    M, K = assemble_1d(uniform_knots(p, N), p)
    V = StencilVectorSpace([N + p] * 3, [p] * 3)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    b = V.zeros().from_numpy(np.ones((N + p,) * 3))
    x = V.zeros()
    monkeypatch.setenv("POMS_PCG_SPEC", "1")
    monkeypatch.setenv("POMS_PCG_GRAPH", "1")
    A.timing(True)
    for _ in range(3):
        x._data.zero_()
        solvers.pcg(A, solvers.damped_jacobi, b, x0=x, tol=1e-6, maxiter=3, _x0_owned=True)
    st = A.spec_stats
    assert st["calls"] == 3 and st["repeats"] == 0 and st["captures"] == 1 and st["replays"] == 2, st
    t, n, d = A.timing_read("jacobi")
    A.timing(False)
    # the capture's launches (one call: 3 + 1 preconditioner calls of 8 sweep launches),
    # their events holding the last replay's times
    assert n == 4 * 8 and t > 0


def test_op_timing_counts_native_launches(gpu):
    """poms_op_timing records every operator launch, including the native loop's."""
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, 16
    M, K = assemble_1d(uniform_knots(p, N), p)
    V = StencilVectorSpace([N + p] * 3, [p] * 3)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    b = V.zeros().from_numpy(np.ones((N + p,) * 3))
    A.timing(True)
    solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=3)
    A.timing(False)
    t, n, d = A.timing_read("jacobi")
    # 3 + 1 preconditioner calls, each from-zero (1 launch) + 8 sweeps
    assert n == 4 * 8 and d == n * (N + p) ** 3 and t > 0
    ta, na, _ = A.timing_read("apply_dot")
    assert na == 3
    A.timing(True, "jacobi", every=4, reserve=16)   # a sample of one epilogue
    solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=3)
    assert A.timing_read("jacobi")[1] == 8 and A.timing_read("apply_dot")[1] == 0
    A.timing(False)

"""Parity at BASELINE.json's full sizes through size-independent properties.

The oracle cannot run at 515^3, so these checks use identities whose expected
value is cheap to form exactly:

* separable inputs x = u0 ⊗ u1 ⊗ u2: A x is a sum of four separable tensors
  built from 1D band products (c Mu⊗Mv⊗Mw + Ku⊗Mv⊗Mw + Mu⊗Kv⊗Mw + Mu⊗Mv⊗Kw);
  the Jacobi sweep's diag(A) is separable the same way;
* symmetry of A: x·(Ay) == y·(Ax) for random x, y.

The expected tensors are formed with torch fp64 outer products on the device
(test plumbing only; the operator itself runs through libpoms_hip.so).
"""
import numpy as np
import pytest
import torch

from poms_amd.splines import assemble_1d, band_to_dense, uniform_knots

pytestmark = pytest.mark.gpu

CONFIGS = {                       # BASELINE.json configs[1..4]
    "2d_p3_1024": (2, 3, 1024),
    "3d_p2_256": (3, 2, 256),
    "3d_p5_256": (3, 5, 256),
    "3d_p3_512": (3, 3, 512),
}


def outer(vs):
    t = vs[0]
    for v in vs[1:]:
        t = torch.einsum("...i,j->...ij", t, v)
    return t


def setup(ndim, p, N, variant=None, align=False):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * ndim, [p] * ndim, align=align)
    A = KronOperator.laplace(V, [M] * ndim, [K] * ndim)
    if variant is not None:
        A.set_variant(variant)
    return V, A, M, K, n


def separable_image(vs, M, K, dev):
    Md, Kd = band_to_dense(M), band_to_dense(K)
    Mv = [torch.from_numpy(Md @ v).to(dev) for v in vs]
    Kv = [torch.from_numpy(Kd @ v).to(dev) for v in vs]
    y = outer(Mv)
    for d in range(len(vs)):
        y += outer([Kv[e] if e == d else Mv[e] for e in range(len(vs))])
    return y


def trel(a, b):
    return float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("align", [False, True])
def test_separable_apply_residual_jacobi_full_size(gpu, cfg, align):
    ndim, p, N = CONFIGS[cfg]
    V, A, M, K, n = setup(ndim, p, N, align=align)
    rng = np.random.default_rng(N + p)
    us = [rng.uniform(-1, 1, n) for _ in range(ndim)]
    ws = [rng.uniform(-1, 1, n) for _ in range(ndim)]
    dev = gpu
    x, b = V.zeros(), V.zeros()
    V.interior(x._data).copy_(outer([torch.from_numpy(u).to(dev) for u in us]))
    V.interior(b._data).copy_(outer([torch.from_numpy(w).to(dev) for w in ws]))
    x._mark_written(), b._mark_written()
    want = separable_image(us, M, K, dev)
    y = A.dot(x)
    assert trel(V.interior(y._data), want) <= 1e-13
    del y
    r = A.residual(b, x)
    want = V.interior(b._data) - want          # b - A x
    assert trel(V.interior(r._data), want) <= 1e-13
    del r
    dM = torch.from_numpy(M[:, p].copy()).to(dev)
    dK = torch.from_numpy(K[:, p].copy()).to(dev)
    D = outer([dM] * ndim)
    for d in range(ndim):
        D += outer([dK if e == d else dM for e in range(ndim)])
    want.mul_(2.0 / 3.0).div_(D)               # dr
    del D
    xo = V.zeros()
    nrm = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
    dr_norm = float(torch.sum(want * want))
    assert abs(nrm - dr_norm) <= 1e-12 * dr_norm
    want.add_(V.interior(x._data))
    assert trel(V.interior(xo._data), want) <= 1e-13
    # the ghost cells of every output stay zero
    xo_g = xo._data.clone()
    V.interior(xo_g).zero_()
    assert not bool(xo_g.any())


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("align", [False, True])
def test_symmetry_full_size(gpu, cfg, align):
    ndim, p, N = CONFIGS[cfg]
    V, A, M, K, n = setup(ndim, p, N, align=align)
    x, y = V.zeros(), V.zeros()
    g = torch.Generator(device=gpu).manual_seed(5)
    V.interior(x._data).uniform_(-1, 1, generator=g)
    V.interior(y._data).uniform_(-1, 1, generator=g)
    x._mark_written(), y._mark_written()
    ax, ay = A.dot(x), A.dot(y)
    s1, s2 = x.dot(ay), y.dot(ax)
    assert abs(s1 - s2) <= 1e-12 * abs(s1)
    # linearity: A(2x - 3y) == 2Ax - 3Ay
    z = x * 2.0 - y * 3.0
    az = A.dot(z)
    want = 2.0 * V.interior(ax._data) - 3.0 * V.interior(ay._data)
    assert trel(V.interior(az._data), want) <= 1e-14


@pytest.mark.parametrize("cfg", ["2d_p3_1024", "3d_p5_256"])
def test_variants_agree_full_size(gpu, cfg):
    """Every kernel variant computes the same operator on the full-size grids."""
    ndim, p, N = CONFIGS[cfg]
    V, A, M, K, n = setup(ndim, p, N)
    x = V.zeros()
    g = torch.Generator(device=gpu).manual_seed(9)
    V.interior(x._data).uniform_(-1, 1, generator=g)
    x._mark_written()
    A.set_variant(0)
    ref = A.dot(x)._data.clone()
    for v in (4, 7, 9, 10):
        A.set_variant(v)
        y = A.dot(x)
        assert trel(y._data, ref) <= 1e-14, v


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("align", [False, True])
def test_bench_kernels_full_size(gpu, cfg, align):
    """Every other kernel the V-cycle bench launches, at the BASELINE sizes (a race
    that only showed at 515^3 has happened on this path before):

    * the two-sweeps-from-zero launch (JACOBI0) == diag_scale then one sweep, which are
      themselves property-checked above; both of its norms;
    * apply + x.Ax (APPLYDOT) == the apply, and its dot == x . (A x);
    * the Jacobi sweep that also forms x_out . b (the JDOT build) == the plain sweep;
    * pcg's fused vector updates (vec_flat_kernel: r -= a q with r.r; x += a p with
      p = s + b p) against torch fp64 on the interiors, ghosts staying zero.
    `sources/solvers.py:103-124, 207-219`."""
    from poms_amd import solvers
    ndim, p, N = CONFIGS[cfg]
    V, A, M, K, n = setup(ndim, p, N, align=align)
    g = torch.Generator(device=gpu).manual_seed(17)
    w = 2.0 / 3.0

    def rnd():
        v = V.zeros()
        V.interior(v._data).uniform_(-1, 1, generator=g)
        v._mark_written()
        return v

    def ghosts_zero(v):
        t = v._data.clone()
        V.interior(t).zero_()
        return not bool(t.any())

    x, b = rnd(), rnd()
    # --- APPLYDOT
    if A.apply_dot_supported:
        q = V.zeros()
        pq = A.dot_inner(x, q)
        y = A.dot(x)
        assert trel(V.interior(q._data), V.interior(y._data)) <= 1e-15
        want = float(torch.sum(V.interior(x._data) * V.interior(y._data)))
        assert abs(pq - want) <= 1e-12 * abs(want)
        assert ghosts_zero(q)
        del q, y
    # --- Jacobi sweep with the fused x_out . b (JDOT) vs the plain sweep
    if A.fused_dot_supported:
        xo1, xo2 = V.zeros(), V.zeros()
        nrm1 = A.jacobi_sweep(b, x, xo1, w, want_norm=True)
        nrm2, xb = A.jacobi_sweep(b, x, xo2, w, want_norm=True, want_dot=True)
        assert trel(V.interior(xo2._data), V.interior(xo1._data)) <= 1e-15
        assert abs(nrm2 - nrm1) <= 1e-12 * nrm1
        want = float(torch.sum(V.interior(xo1._data) * V.interior(b._data)))
        assert abs(xb - want) <= 1e-12 * abs(want)
        assert ghosts_zero(xo2)
        del xo1, xo2
    # --- two sweeps from zero (JACOBI0) vs diag_scale + one sweep
    if A.from_zero_supported:
        y0 = V.zeros()
        n1, n2 = A.jacobi_from_zero(b, y0, w, want_norm=True)
        x1, x2 = V.zeros(), V.zeros()
        m1 = A.diag_scale(b, x1, scale=w, want_norm=True)
        m2 = A.jacobi_sweep(b, x1, x2, w, want_norm=True)
        assert trel(V.interior(y0._data), V.interior(x2._data)) <= 1e-13
        assert abs(n1 - m1) <= 1e-12 * m1 and abs(n2 - m2) <= 1e-12 * m2
        assert ghosts_zero(y0)
        del y0, x1, x2
    # --- pcg vector updates
    r, qv, xs, pv, sv = rnd(), rnd(), rnd(), rnd(), rnd()
    r0, q0 = V.interior(r._data).clone(), V.interior(qv._data).clone()
    alpha, beta = 0.37, -1.25
    rr = solvers._pcg_r_update(V, alpha, r, qv)
    want = r0 - alpha * q0
    assert trel(V.interior(r._data), want) <= 1e-15
    want_rr = float(torch.sum(want * want))
    assert abs(rr - want_rr) <= 1e-12 * want_rr
    assert ghosts_zero(r)
    del r0, q0, want
    x0, p0, s0 = (V.interior(v._data).clone() for v in (xs, pv, sv))
    solvers._pcg_xp_update(V, alpha, beta, xs, pv, sv)
    assert trel(V.interior(xs._data), x0 + alpha * p0) <= 1e-15
    assert trel(V.interior(pv._data), s0 + beta * p0) <= 1e-15
    assert ghosts_zero(xs) and ghosts_zero(pv)

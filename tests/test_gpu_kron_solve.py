"""Kronecker direct solve (GLT preconditioner) on the GPU: the reference's own
outputs (tests/golden/kron_solve.npz, pcg_glt.npz), the oracle on seeded inputs
(pivoting, every band shape up to kl + ku = 16, 1D/2D/3D, both layouts, in place)
and a full-size solve -> apply round trip."""
import numpy as np
import pytest
import torch

from oracle import poms_oracle as orc

pytestmark = pytest.mark.gpu


def load(golden_dir, name):
    z = np.load(golden_dir / name, allow_pickle=False)
    out = {}
    for k in z.files:
        case, field = k.split("__", 1)
        out.setdefault(case, {})[field] = z[k]
    return out


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _interior(X, pads, points):
    return X[tuple(slice(p, p + n) for p, n in zip(pads, points))]


def test_kron_solve_bnd_pyccel_golden(gpu, golden_dir):
    """Host drop-ins of `kron_solve_par_bnd_pyccel_2d/_3d` and `kron_solve_serial_pyccel_2d`
    == the reference kernels' outputs (`pyccel/pyccel_functions.py:26-248`)."""
    from poms_amd.kron_solve import (kron_solve_par_bnd_pyccel_2d, kron_solve_par_bnd_pyccel_3d,
                                     kron_solve_serial_pyccel_2d, to_bnd)
    for name, c in load(golden_dir, "kron_solve.npz").items():
        if name == "spl_wrappers":
            continue
        pts, pads = [int(v) for v in c["points"]], [int(v) for v in c["pads"]]
        Y = np.ascontiguousarray(c["Y"])
        X = np.full_like(Y, 7.0)             # ghosts must survive
        bands = []
        for d in range(len(pts)):
            bands += list(to_bnd(c[f"A{d + 1}"]))
        if len(pts) == 2:
            kron_solve_par_bnd_pyccel_2d(*bands, X, Y, pts, pads)
        else:
            kron_solve_par_bnd_pyccel_3d(*bands, X, Y, pts, pads)
        want = _interior(c["X_bnd"], pads, pts)
        assert rel(_interior(X, pads, pts), want) <= 1e-13, name
        ghost = X.copy()
        _interior(ghost, pads, pts)[...] = 7.0
        assert np.all(ghost == 7.0), name
        if "X_serial" in c:
            Xs = np.zeros_like(Y)
            kron_solve_serial_pyccel_2d(c["A1"], c["A2"], Xs, Y, pts, pads)
            assert rel(_interior(Xs, pads, pts), _interior(c["X_serial"], pads, pts)) <= 1e-13, name


def test_kron_solve_spl_wrappers_golden(gpu, golden_dir):
    """`kron_solve_serial` / `kron_solve_par` (`sources/kron_product.py:93-158`) on device vectors."""
    from poms_amd.kron_solve import kron_solve_par, kron_solve_serial
    from poms_amd.stencil import StencilVectorSpace
    c = load(golden_dir, "kron_solve.npz")["spl_wrappers"]
    pts, pads = [int(v) for v in c["points"]], [int(v) for v in c["pads"]]
    V = StencilVectorSpace(pts, pads)
    Y = V.zeros().from_numpy(_interior(c["Y"], pads, pts))
    assert rel(kron_solve_serial(c["A1"], c["A2"], Y).to_local_numpy(), _interior(c["X_serial"], pads, pts)) <= 1e-13
    assert rel(kron_solve_par(c["A1"], c["A2"], Y).to_local_numpy(), _interior(c["X_par"], pads, pts)) <= 1e-13


def test_pivots_match_scipy_dgbtrf(gpu):
    from scipy.linalg.lapack import dgbtrf
    from poms_amd.kron_solve import KronSolver, to_bnd
    from poms_amd.stencil import StencilVectorSpace
    rng = np.random.default_rng(5)
    F = [np.triu(np.tril(rng.uniform(-1, 1, (m, m)), ku), -kl) for m, kl, ku in ((30, 4, 2), (25, 2, 5))]
    ks = KronSolver(StencilVectorSpace([30, 25], [2, 2]), F)
    assert ks.info == (0, 0)
    for d in range(2):
        ab, la, ua = to_bnd(F[d])
        _, piv, _ = dgbtrf(ab, la, ua)
        np.testing.assert_array_equal(ks.pivots(d), piv)


def _band(rng, m, kl, ku, boost=0.0):
    return np.triu(np.tril(rng.uniform(-1, 1, (m, m)), ku), -kl) + boost * np.eye(m)


CASES = [
    # (shape, pads, [(kl, ku) per axis], align)
    ((37,), (2,), [(1, 1)], False),
    ((50, 41), (3, 3), [(2, 2), (3, 1)], False),
    ((64, 70), (3, 3), [(1, 4), (5, 5)], True),
    ((24, 19, 33), (2, 2, 2), [(2, 1), (1, 2), (3, 3)], False),
    ((21, 30, 47), (3, 3, 3), [(8, 8), (4, 4), (6, 2)], True),
    ((9, 12, 130), (1, 1, 1), [(0, 0), (0, 3), (3, 0)], False),
    ((17, 16, 16), (5, 5, 5), [(5, 5), (8, 7), (2, 6)], False),
]


@pytest.mark.parametrize("shape,pads,bw,align", CASES)
@pytest.mark.parametrize("inplace", [False, True])
def test_kron_solve_vs_oracle(gpu, shape, pads, bw, align, inplace):
    from poms_amd.kron_solve import KronSolver
    from poms_amd.stencil import StencilVectorSpace
    rng = np.random.default_rng(sum(shape) + 7 * len(shape))
    F = [_band(rng, m, kl, ku, boost=0.5) for m, (kl, ku) in zip(shape, bw)]
    yg = rng.standard_normal(shape)
    V = StencilVectorSpace(list(shape), list(pads), align=align)
    ks = KronSolver(V, F)
    y = V.zeros().from_numpy(yg)
    ref = orc.kron_solve(F, yg)
    x = ks.solve(y, out=y if inplace else None)
    assert rel(x.to_local_numpy(), ref) <= 1e-12
    # ghosts stay zero
    full = x._data.cpu().numpy()
    inner = _interior(full, pads, shape).copy()
    _interior(full, pads, shape)[...] = 0.0
    assert not np.any(full)
    assert np.isfinite(inner).all()


def test_singular_factor_fails_loudly(gpu):
    from poms_amd._lib import PomsError
    from poms_amd.kron_solve import KronSolver
    from poms_amd.stencil import StencilVectorSpace
    A = np.eye(6)
    A[3, 3] = 0.0
    ks = KronSolver(StencilVectorSpace([6, 5], [1, 1]), [A, np.eye(5)])
    assert ks.info == (4, 0)
    V = ks.V
    with pytest.raises(PomsError):
        ks.solve(V.zeros())


def _glt_space(p, ne):
    from poms_amd.splines import assemble_1d, make_open_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M, K = assemble_1d(make_open_knots(p, ne + p), p)
    n = ne + p
    V = StencilVectorSpace([n, n], [p, p])
    return V, KronOperator.laplace(V, [M, M], [K, K]), M, K


@pytest.mark.parametrize("case", ["p1_ne4", "p2_ne8", "p3_ne8", "p3_ne12"])
def test_pcg_glt_golden(gpu, golden_dir, case):
    """`pcg_glt` (`sources/solvers.py:239-306`) == the reference's iterates and info."""
    from poms_amd.solvers import pcg_glt
    from tests.test_kron_solve_oracle import glt_bound
    c = load(golden_dir, "pcg_glt.npz")[case]
    p, ne = int(c["p"]), int(c["ne"])
    V, A, M, K = _glt_space(p, ne)
    n = ne + p
    b = V.zeros().from_numpy(c["b"].reshape(n, n))
    x, info = pcg_glt(A, c["M1"], c["M2"], b, tol=1e-8, maxiter=100)
    assert info["niter"] == int(c["glt_test_info"][0])
    assert info["success"] == bool(c["glt_test_info"][1])
    apply = lambda v: orc.kron_sum_apply(v.reshape(n, n), [M, M], [K, K]).reshape(-1)
    assert rel(x.toarray(), c["glt_test"]) <= glt_bound(c, apply)
    for m in (1, 3):
        x, info = pcg_glt(A, c["M1"], c["M2"], b, tol=0.0, maxiter=m)
        assert info["niter"] == int(c[f"glt_m{m}_tol0_info"][0])
        assert rel(x.toarray(), c[f"glt_m{m}_tol0"]) <= 1e-9
    ones = V.zeros().from_numpy(np.ones((n, n)))
    x0 = V.zeros().from_numpy(c["glt_post_x0"].reshape(n, n))
    x, info = pcg_glt(A, c["M1"], c["M2"], ones, x0=x0, tol=1e-6, maxiter=p + 1)
    assert info["niter"] == int(c["glt_post_info"][0])
    assert rel(x.toarray(), c["glt_post"]) <= 1e-9


@pytest.mark.parametrize("n,p", [(258, 3), (515, 3)])
def test_kron_solve_full_size_round_trip(gpu, n, p):
    """Solve with the p-degree collocation factors on a BASELINE-size grid, then apply
    the same Kronecker product with the operator kernels: Y comes back (size-
    independent property; the Kron solve is exact up to rounding)."""
    from poms_amd.kron_solve import KronSolver
    from poms_amd.splines import collocation_cardinal_splines, dense_to_band
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    C = collocation_cardinal_splines(p, n)
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    ks = KronSolver(V, [C, C, C])
    g = torch.Generator(device=gpu).manual_seed(3)
    y = V.zeros()
    V.interior(y._data).copy_(torch.rand(V.local_npts, generator=g, device=gpu, dtype=torch.float64) * 2 - 1)
    x = ks.solve(y)
    op = KronOperator.product(V, [dense_to_band(C, p)] * 3)
    y2 = op.dot(x)
    a, b = V.interior(y2._data), V.interior(y._data)
    assert float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)) <= 1e-13

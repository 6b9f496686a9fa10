"""Kronecker direct solve / GLT smoother: the CPU oracle pinned to the reference's
own outputs (tests/golden/kron_solve.npz, pcg_glt.npz from make_golden.py, which
runs `pyccel/pyccel_functions.py:26-248`, `sources/kron_product.py:93-191` and
`sources/solvers.py:239-306`), plus the host set-up the C-ABI mirrors."""
import numpy as np
import pytest
from scipy.linalg.lapack import dgbtrf

from oracle import poms_oracle as orc



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


def test_kron_solve_oracle_matches_reference(golden_dir):
    cases = load(golden_dir, "kron_solve.npz")
    assert len(cases) >= 9
    for name, c in cases.items():
        if name == "spl_wrappers":
            continue
        pts, pads = [int(v) for v in c["points"]], [int(v) for v in c["pads"]]
        F = [c[f"A{d + 1}"] for d in range(len(pts))]
        Yi = _interior(c["Y"], pads, pts)
        X = orc.kron_solve(F, Yi)
        assert rel(X, _interior(c["X_bnd"], pads, pts)) <= 1e-13, name
        assert rel(X, c["X_kron_ref"]) <= 1e-11, name      # dense kron solve (conditioning)
        if "X_serial" in c:
            assert rel(_interior(c["X_serial"], pads, pts), _interior(c["X_bnd"], pads, pts)) <= 1e-13, name


def test_kron_solve_spl_wrappers(golden_dir):
    c = load(golden_dir, "kron_solve.npz")["spl_wrappers"]
    pts, pads = [int(v) for v in c["points"]], [int(v) for v in c["pads"]]
    X = orc.kron_solve([c["A1"], c["A2"]], _interior(c["Y"], pads, pts))
    assert rel(X, _interior(c["X_serial"], pads, pts)) <= 1e-13
    assert rel(X, _interior(c["X_par"], pads, pts)) <= 1e-13


@pytest.mark.parametrize("n,kl,ku,seed", [(12, 1, 1, 0), (25, 3, 2, 1), (40, 5, 5, 2), (9, 0, 3, 3),
                                          (16, 4, 0, 4), (33, 8, 8, 5)])
def test_gbtrf_pivots_match_lapack(n, kl, ku, seed):
    """The dgbtf2 restatement (oracle and poms_ksolve_create share it) picks scipy's pivots."""
    rng = np.random.default_rng(seed)
    A = np.triu(np.tril(rng.uniform(-1, 1, (n, n)), ku), -kl)
    ab, la, ua = orc.to_bnd(A)
    lu, piv, info = dgbtrf(ab, la, ua)
    lu2, piv2, info2 = orc.gbtrf(ab, la, ua)
    assert info == info2 == 0
    np.testing.assert_array_equal(piv, piv2)
    assert np.max(np.abs(lu - lu2)) <= 1e-12 * np.max(np.abs(lu))
    b = rng.uniform(-1, 1, (n, 4))
    assert rel(orc.gbtrs(lu2, la, ua, piv2, b), np.linalg.solve(A, b)) <= 1e-11


def glt_bound(c, apply):
    """Converged (tol=1e-8, tens of iterations) iterates agree only to the rounding
    spread of the iteration: 20x the distance between two oracle runs whose
    preconditioner differs only in summation order (axis order of the Kron solve)."""
    b = c["b"]
    n = c["M1"].shape[0]
    xa, _ = orc.pcg(apply, lambda r: orc.kron_solve([c["M2"], c["M1"]], r.reshape(n, n)).reshape(-1), b,
                    tol=1e-8, maxiter=100)
    xb, _ = orc.pcg(apply, lambda r: np.ascontiguousarray(
        orc.kron_solve([c["M1"], c["M2"]], r.reshape(n, n).T).T).reshape(-1), b, tol=1e-8, maxiter=100)
    return max(1e-9, 20 * rel(xa, xb))


def test_pcg_glt_oracle_matches_reference(golden_dir):
    from poms_amd.splines import assemble_1d, make_open_knots
    for name, c in load(golden_dir, "pcg_glt.npz").items():
        p, ne = int(c["p"]), int(c["ne"])
        M, K = assemble_1d(make_open_knots(p, ne + p), p)
        n = ne + p
        apply = lambda v: orc.kron_sum_apply(v.reshape(n, n), [M, M], [K, K]).reshape(-1)
        F = [c["M2"], c["M1"]]
        b = c["b"]
        x, info = orc.pcg_glt(apply, F, b, tol=1e-8, maxiter=100)
        ref = c["glt_test_info"]
        assert info["niter"] == int(ref[0]) and info["success"] == bool(ref[1]), name
        assert rel(x, c["glt_test"]) <= glt_bound(c, apply), name
        for m in (1, 3):
            x, info = orc.pcg_glt(apply, F, b, tol=0.0, maxiter=m)
            assert info["niter"] == int(c[f"glt_m{m}_tol0_info"][0]), name
            assert rel(x, c[f"glt_m{m}_tol0"]) <= 1e-9, name
        ones = np.ones(n * n)
        x, info = orc.pcg_glt(apply, F, ones, x0=c["glt_post_x0"], tol=1e-6, maxiter=p + 1)
        assert info["niter"] == int(c["glt_post_info"][0]), name
        assert rel(x, c["glt_post"]) <= 1e-9, name


def test_collocation_cardinal_splines_restatement():
    """Known cardinal-spline values (spl absent: the restatement is pinned by these)."""
    from poms_amd.splines import collocation_cardinal_splines
    C3 = collocation_cardinal_splines(3, 6)
    assert np.allclose(C3[2, 1:4], [1 / 6, 4 / 6, 1 / 6], rtol=0, atol=1e-15)
    C2 = collocation_cardinal_splines(2, 6)
    assert np.allclose(C2[2, 1:4], [1 / 8, 6 / 8, 1 / 8], rtol=0, atol=1e-15)
    assert np.array_equal(collocation_cardinal_splines(1, 5), np.eye(5))
    C5 = collocation_cardinal_splines(5, 9)
    assert np.allclose(C5[4, 2:7], np.array([1, 26, 66, 26, 1]) / 120, rtol=0, atol=1e-15)
    for p in (1, 2, 3, 4, 5):   # partition of unity on the interior rows, symmetry
        C = collocation_cardinal_splines(p, 3 * p + 3)
        assert np.allclose(C.sum(axis=1)[p:-p], 1.0, atol=1e-14)
        assert np.array_equal(C, C.T)
        assert np.array_equal(C, orc.collocation_cardinal_splines(p, 3 * p + 3))


def test_assembly_varcoef_oracle_matches_reference(golden_dir):
    """The d-dimensional quadrature-assembly restatement (a = c = 1) == the reference's
    own `assembly_2d` stencils (`sources/matrix_assembler.py:84-179`)."""
    from oracle import spl_standin as S
    for name, c in load(golden_dir, "assembly_2d.npz").items():
        p = int(c["p"])
        ne = [int(v) for v in c["ne"]]
        T = [S.make_open_knots(p, e + p) for e in ne]
        o = orc.assembly_varcoef(T, [p, p])
        assert np.max(np.abs(o - c["stencil"])) <= 1e-14 * np.max(np.abs(c["stencil"])), name

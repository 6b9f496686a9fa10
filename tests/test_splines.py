"""Host-side spline set-up (poms_amd.splines): known answers and structural properties.

The 1D factors are the only input of every device operator, so they are pinned
independently of the reference: interior rows of the uniform mass/stiffness
matrices are samples of the centred cardinal B-spline of degree 2p+1 and of its
second derivative (exact rational arithmetic below); row sums, symmetry,
quadrature exactness and the nested-space Galerkin identity P^T M_f P = M_c
close the rest.  The knot-insertion matrix is pinned by spline reproduction.
"""
from fractions import Fraction
from math import comb, factorial

import numpy as np
import pytest

from poms_amd.splines import (assemble_1d, band_to_dense, basis_funs_ders, dense_to_band, find_span,
                              greville, insert_knot_matrix, make_open_knots, matrix_multi_stages,
                              uniform_knots)
from poms_amd.multilevels import knots_to_insert


def cardinal(m: int, x: Fraction, deriv: int = 0) -> Fraction:
    """Centred cardinal B-spline of degree m (support [-(m+1)/2, (m+1)/2]) or its derivative."""
    s = Fraction(0)
    e = m - deriv
    for j in range(m + 2):
        t = x + Fraction(m + 1, 2) - j
        if t > 0:
            s += (-1) ** j * comb(m + 1, j) * t ** e
    return s / factorial(e)


def spline_eval(T, p, c, x):
    span = find_span(T, p, x)
    D = basis_funs_ders(T, p, x, span, 0)
    return float(D[0] @ c[span - p:span + 1])


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5])
def test_uniform_interior_rows_known_answer(p):
    N = 6 * p + 4
    h = 1.0 / N
    M, K = assemble_1d(uniform_knots(p, N), p)
    i = (N + p) // 2
    m = 2 * p + 1
    for k in range(2 * p + 1):
        off = Fraction(k - p)
        assert abs(M[i, k] - h * float(cardinal(m, off))) <= 1e-15, (p, k)
        assert abs(K[i, k] + float(cardinal(m, off, 2)) / h) <= 1e-11 / h, (p, k)


@pytest.mark.parametrize("p", [1, 2, 3, 5])
@pytest.mark.parametrize("knots", ["uniform", "graded"])
def test_factor_structure(p, knots):
    N = 13
    if knots == "uniform":
        T = uniform_knots(p, N)
    else:
        inner = np.sort(np.random.default_rng(p).uniform(0.02, 0.98, N - 1))
        T = np.concatenate([np.zeros(p + 1), inner, np.ones(p + 1)])
    n = len(T) - p - 1
    M, K = assemble_1d(T, p)
    Md, Kd = band_to_dense(M), band_to_dense(K)
    np.testing.assert_allclose(Md, Md.T, atol=1e-15)
    np.testing.assert_allclose(Kd, Kd.T, atol=1e-10 * np.abs(Kd).max())
    # integral of B_i and of its derivative
    np.testing.assert_allclose(M.sum(1), (T[p + 1:p + 1 + n] - T[:n]) / (p + 1), rtol=1e-13, atol=1e-16)
    assert np.abs(K.sum(1)).max() <= 1e-11 * np.abs(K).max()
    # p+1 Gauss points are exact for the degree-2p integrands
    M2, K2 = assemble_1d(T, p, nquad=p + 3)
    np.testing.assert_allclose(M2, M, atol=1e-15)
    np.testing.assert_allclose(K2, K, atol=1e-10 * np.abs(K).max())
    # SPD
    assert np.linalg.eigvalsh(Md).min() > 0
    assert np.linalg.eigvalsh(Kd + Md).min() > 0
    np.testing.assert_array_equal(dense_to_band(Md, p), M)


@pytest.mark.parametrize("p", [1, 2, 3, 4])
def test_basis_partition_of_unity_and_derivative(p):
    T = uniform_knots(p, 9)
    rng = np.random.default_rng(0)
    for x in rng.uniform(0, 1, 20):
        span = find_span(T, p, x)
        assert T[span] <= x < T[span + 1]
        D = basis_funs_ders(T, p, x, span, 1)
        assert abs(D[0].sum() - 1.0) <= 1e-14
        assert abs(D[1].sum()) <= 1e-11
        eps = 1e-6
        Dp = basis_funs_ders(T, p, x + eps, span, 0)[0]
        Dm = basis_funs_ders(T, p, x - eps, span, 0)[0]
        np.testing.assert_allclose(D[1], (Dp - Dm) / (2 * eps), atol=1e-5)
    assert find_span(T, p, 1.0) == len(T) - p - 2


@pytest.mark.parametrize("p", [1, 2, 3, 4])
@pytest.mark.parametrize("nc,nf", [(4, 8), (8, 32), (3, 9)])
def test_multi_stage_prolongation(p, nc, nf):
    """P1 reproduces coarse splines exactly and is a partition of unity (`sources/mg_jac.py:64-70`)."""
    Tc, Tf = uniform_knots(p, nc), uniform_knots(p, nf)
    ncb, nfb = len(Tc) - p - 1, len(Tf) - p - 1
    ts = knots_to_insert(Tf, nfb, p, Tc, ncb, p)
    P1 = matrix_multi_stages(ts, ncb, p, Tc)
    assert P1.shape == (nfb, ncb)
    np.testing.assert_allclose(P1.sum(1), 1.0, atol=1e-14)
    assert P1.min() >= -1e-15
    c = np.random.default_rng(1).standard_normal(ncb)
    cf = P1 @ c
    for x in np.linspace(0, 1, 37):
        assert abs(spline_eval(Tc, p, c, x) - spline_eval(Tf, p, cf, x)) <= 1e-12
    # Greville abscissae of the fine space reproduce the identity function too
    np.testing.assert_allclose(P1 @ greville(Tc, p), greville(Tf, p), atol=1e-14)
    # nested spaces: Galerkin coarse operators are the coarse-space matrices
    if nf % nc == 0:
        Mc, Kc = (band_to_dense(F) for F in assemble_1d(Tc, p))
        Mf, Kf = (band_to_dense(F) for F in assemble_1d(Tf, p))
        np.testing.assert_allclose(P1.T @ Mf @ P1, Mc, atol=1e-14)
        np.testing.assert_allclose(P1.T @ Kf @ P1, Kc, atol=1e-10 * np.abs(Kc).max())


def test_single_knot_insertion():
    p = 2
    T = make_open_knots(p, 5)
    A, Tn = insert_knot_matrix(T, p, 0.3)
    assert A.shape == (6, 5) and len(Tn) == len(T) + 1
    np.testing.assert_allclose(A.sum(1), 1.0, atol=1e-15)
    assert np.all(np.diff(Tn) >= 0) and 0.3 in Tn


def test_make_open_knots_convention():
    """spl's make_open_knots(p, n) takes the number of basis functions (`sources/mg_jac.py:28`)."""
    T = make_open_knots(3, 8)
    assert len(T) == 8 + 3 + 1
    np.testing.assert_array_equal(T[:4], 0.0)
    np.testing.assert_array_equal(T[-4:], 1.0)
    np.testing.assert_allclose(T[4:8], [0.2, 0.4, 0.6, 0.8])
    with pytest.raises(ValueError):
        make_open_knots(3, 3)

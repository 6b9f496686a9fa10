"""Host-side B-spline setup: knot vectors, 1D mass/stiffness factors, knot insertion.

This is set-up code that runs once per operator (the reference calls it
"assembly", `sources/matrix_assembler.py:10-253`, and it is not on the timed
path).  It produces the two banded 1D factors from which every operator of the
hot path is built:

    M[i, j] = \\int B_i B_j dx          (mass)
    K[i, j] = \\int B_i' B_j' dx        (stiffness)

The reference assembles the 2D `-Δu + u` stencil directly
(`sources/matrix_assembler.py:173`: ``(bi0*bj0 + bix*bjx + biy*bjy)*wvol``);
that integrand factorises exactly into ``M⊗M + K⊗M + M⊗K`` which is what the
device kernels apply in sum-factorised form.

Band storage convention (shared with the C-ABI, see ``include/poms_hip.h``):
``F_band[i, k] = F[i, i + k - p]`` for ``k = 0 .. 2p``, zero where
``i + k - p`` falls outside ``[0, n)`` -- the 1D ``StencilMatrix`` layout of
spl (``M[i, k]`` with ``k`` offset by ``p``) used by
`pyccel/pyccel_functions.py:4-21` (``A[i1, k]``, ``k in range(2*p1+1)``).

Knot conventions follow spl as used by the reference:
``make_open_knots(p, n)`` takes the number of basis functions ``n`` and
returns ``n + p + 1`` open knots on [0, 1] (`sources/mg_jac.py:28-29`,
`sources/multilevels.py:12-33` iterate ``range(pf+1, nf)`` over the interior
knots).  A grid of ``N`` cells therefore has ``n = N + p`` basis functions.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "make_open_knots", "uniform_knots", "find_span", "basis_funs_ders",
    "assemble_1d", "band_to_dense", "dense_to_band", "insert_knot_matrix",
    "matrix_multi_stages", "greville",
]


def make_open_knots(p: int, n: int) -> np.ndarray:
    """Open uniform knot vector with ``n`` basis functions of degree ``p``.

    Mirrors spl's ``make_open_knots(p, n)`` as called at `sources/mg_jac.py:28`.
    """
    if n < p + 1:
        raise ValueError(f"need n >= p+1 basis functions, got n={n}, p={p}")
    ncells = n - p
    interior = np.arange(1, ncells, dtype=np.float64) / ncells
    return np.concatenate([np.zeros(p + 1), interior, np.ones(p + 1)])


def uniform_knots(p: int, ncells: int) -> np.ndarray:
    """Open uniform knots on [0, 1] with ``ncells`` cells (``n = ncells + p``)."""
    return make_open_knots(p, ncells + p)


def find_span(T: np.ndarray, p: int, x: float) -> int:
    """Index ``i`` with ``T[i] <= x < T[i+1]`` and ``p <= i <= n-1``."""
    n = len(T) - p - 1
    if x >= T[n]:
        return n - 1
    lo, hi = p, n
    # binary search on the non-decreasing knot vector
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if x < T[mid]:
            hi = mid
        else:
            lo = mid
    return lo


def basis_funs_ders(T: np.ndarray, p: int, x: float, span: int, nders: int) -> np.ndarray:
    """Values and derivatives of the ``p+1`` B-splines that are non-zero at ``x``.

    Returns ``D`` of shape ``(nders+1, p+1)``; ``D[d, j]`` is the ``d``-th
    derivative of ``B_{span-p+j}`` at ``x`` (Cox-de Boor triangle with
    derivative recursion).
    """
    ndu = np.zeros((p + 1, p + 1))
    left = np.zeros(p + 1)
    right = np.zeros(p + 1)
    ndu[0, 0] = 1.0
    for j in range(1, p + 1):
        left[j] = x - T[span + 1 - j]
        right[j] = T[span + j] - x
        saved = 0.0
        for r in range(j):
            # lower triangle keeps knot differences, upper keeps basis values
            ndu[j, r] = right[r + 1] + left[j - r]
            tmp = ndu[r, j - 1] / ndu[j, r]
            ndu[r, j] = saved + right[r + 1] * tmp
            saved = left[j - r] * tmp
        ndu[j, j] = saved
    ders = np.zeros((nders + 1, p + 1))
    ders[0, :] = ndu[:, p]
    a = np.zeros((2, p + 1))
    for r in range(p + 1):
        s1, s2 = 0, 1
        a[0, 0] = 1.0
        for k in range(1, nders + 1):
            d = 0.0
            rk, pk = r - k, p - k
            if r >= k:
                a[s2, 0] = a[s1, 0] / ndu[pk + 1, rk]
                d = a[s2, 0] * ndu[rk, pk]
            j1 = 1 if rk >= -1 else -rk
            j2 = k - 1 if r - 1 <= pk else p - r
            for j in range(j1, j2 + 1):
                a[s2, j] = (a[s1, j] - a[s1, j - 1]) / ndu[pk + 1, rk + j]
                d += a[s2, j] * ndu[rk + j, pk]
            if r <= pk:
                a[s2, k] = -a[s1, k - 1] / ndu[pk + 1, r]
                d += a[s2, k] * ndu[r, pk]
            ders[k, r] = d
            s1, s2 = s2, s1
    fac = float(p)
    for k in range(1, nders + 1):
        ders[k, :] *= fac
        fac *= (p - k)
    return ders


def assemble_1d(T: np.ndarray, p: int, nquad: int | None = None, canonical: bool = True):
    """Banded 1D mass and stiffness factors ``(M_band, K_band)``, each ``(n, 2p+1)``.

    Element loop over non-empty knot spans with ``nquad`` (default ``p+1``)
    Gauss-Legendre points per element -- the quadrature the reference's
    ``assembly_1d``/``assembly_2d`` use (`sources/matrix_assembler.py:46-73`,
    ``k1 = V.quad_order``), exact for the degree-2p integrands.

    ``canonical``: on uniform open knots every row in ``[2p, n - 2p)`` is the
    same symmetric (Toeplitz) row mathematically, but the element loop leaves
    rounding differences of a few ulp between rows.  Those rows are set to the
    symmetrised middle row so the device kernels recognise the Toeplitz
    interior bitwise (``poms_op_create``) and use their pair-sum fast paths.
    The change is at the 1e-16 level (the golden-vector tests hold either way).
    """
    T = np.asarray(T, dtype=np.float64)
    n = len(T) - p - 1
    nq = p + 1 if nquad is None else int(nquad)
    xg, wg = np.polynomial.legendre.leggauss(nq)
    M = np.zeros((n, 2 * p + 1))
    K = np.zeros((n, 2 * p + 1))
    for span in range(p, n):
        a, b = T[span], T[span + 1]
        if b <= a:
            continue
        half = 0.5 * (b - a)
        for g in range(nq):
            x = a + half * (xg[g] + 1.0)
            w = half * wg[g]
            D = basis_funs_ders(T, p, x, span, 1)
            for il in range(p + 1):
                i = span - p + il
                for jl in range(p + 1):
                    j = span - p + jl
                    k = j - i + p
                    M[i, k] += D[0, il] * D[0, jl] * w
                    K[i, k] += D[1, il] * D[1, jl] * w
    if canonical and _uniform_interior(T, p) and n - 2 * p > 2 * p:
        # the interior rows are samples of the centred cardinal B-spline of degree 2p+1
        # (mass, times h) and of minus its second derivative (stiffness, over h): exact
        # rationals, rounded once -- closer to the true integrals than any assembled row
        h = float(np.unique(T)[1] - np.unique(T)[0])
        cm, ck = _cardinal_rows(p)
        M[2 * p:n - 2 * p] = h * cm
        K[2 * p:n - 2 * p] = -ck / h
    return M, K


_CARD: dict = {}


def _cardinal_rows(p: int):
    """Interior band rows of the uniform mass (/h) and second-derivative (*h) matrices."""
    if p not in _CARD:
        from fractions import Fraction
        from math import comb, factorial
        m = 2 * p + 1

        def card(x, deriv):
            e = m - deriv
            acc = Fraction(0)
            for j in range(m + 2):
                t = x + Fraction(m + 1, 2) - j
                if t > 0:
                    acc += (-1) ** j * comb(m + 1, j) * t ** e
            return acc / factorial(e)

        _CARD[p] = (np.array([float(card(Fraction(k - p), 0)) for k in range(2 * p + 1)]),
                    np.array([float(card(Fraction(k - p), 2)) for k in range(2 * p + 1)]))
    return _CARD[p]


def _uniform_interior(T: np.ndarray, p: int) -> bool:
    """Open knot vector whose non-empty spans all have one length (to 1e-12)."""
    inner = np.unique(np.asarray(T, dtype=np.float64))
    if len(inner) < 3:
        return False
    d = np.diff(inner)
    return bool(np.all(np.abs(d - d[0]) <= 1e-12 * d[0]))


def band_to_dense(band: np.ndarray) -> np.ndarray:
    """Dense ``(n, n)`` matrix from ``(n, 2p+1)`` band rows."""
    n, w = band.shape
    p = (w - 1) // 2
    A = np.zeros((n, n))
    for i in range(n):
        for k in range(w):
            j = i + k - p
            if 0 <= j < n:
                A[i, j] = band[i, k]
    return A


def dense_to_band(A: np.ndarray, p: int) -> np.ndarray:
    """``(n, 2p+1)`` band rows of a square matrix (entries outside the band dropped)."""
    n = A.shape[0]
    band = np.zeros((n, 2 * p + 1))
    for i in range(n):
        for k in range(2 * p + 1):
            j = i + k - p
            if 0 <= j < n:
                band[i, k] = A[i, j]
    return band


def insert_knot_matrix(T: np.ndarray, p: int, t: float):
    """Boehm single-knot insertion: returns ``(A, T_new)`` with ``A`` of shape ``(n+1, n)``.

    Coefficients of a spline on ``T`` map to the refined knot vector by
    ``c_new = A @ c`` (``A[i, i] = alpha_i``, ``A[i, i-1] = 1 - alpha_i``).
    """
    T = np.asarray(T, dtype=np.float64)
    n = len(T) - p - 1
    k = find_span(T, p, t)
    A = np.zeros((n + 1, n))
    for i in range(n + 1):
        if i <= k - p:
            alpha = 1.0
        elif i >= k + 1:
            alpha = 0.0
        else:
            alpha = (t - T[i]) / (T[i + p] - T[i])
        if i < n:
            A[i, i] += alpha
        if i >= 1:
            A[i, i - 1] += 1.0 - alpha
    T_new = np.concatenate([T[: k + 1], [t], T[k + 1:]])
    return A, T_new


def matrix_multi_stages(ts, n: int, p: int, knots) -> np.ndarray:
    """Prolongation ``P1`` (``n_f x n_c``) inserting all knots ``ts`` into ``knots``.

    Restatement of spl's ``matrix_multi_stages(Ts, nc, p, Tc)`` as used by the
    V-cycle driver (`sources/mg_jac.py:67-70`: ``R1 = P1.T``, ``P = kron(P1, P1)``
    acting on coarse coefficients).  spl's own source is not available here;
    the matrix is pinned by spline reproduction (coarse spline == fine spline
    with ``P1 @ c`` coefficients) and partition of unity (rows sum to 1).
    """
    T = np.asarray(knots, dtype=np.float64)
    if len(T) != n + p + 1:
        raise ValueError("knot vector length does not match n + p + 1")
    P = np.eye(n)
    for t in sorted(np.asarray(ts, dtype=np.float64)):
        A, T = insert_knot_matrix(T, p, float(t))
        P = A @ P
    return P


def greville(T: np.ndarray, p: int) -> np.ndarray:
    """Greville abscissae (knot averages) -- used by the spline-reproduction tests."""
    n = len(T) - p - 1
    return np.array([np.mean(T[i + 1:i + p + 1]) if p > 0 else T[i] for i in range(n)])


def cardinal_bspline(p: int, x):
    """Cardinal B-spline of degree p on the integer knots 0..p+1 (truncated-power form)."""
    from math import comb, factorial
    x = np.asarray(x, dtype=np.float64)
    s = np.zeros_like(x)
    for k in range(p + 2):
        s += (-1) ** k * comb(p + 1, k) * np.where(x > k, (x - k) ** p, 0.0)
    return np.where((x > 0) & (x < p + 1), s / factorial(p), 0.0)


def collocation_cardinal_splines(p: int, n: int) -> np.ndarray:
    """The GLT preconditioner's 1D matrix (`sources/mg_glt.py:115-116`): spl's
    ``collocation_cardinal_splines(p, n)``, restated because spl is absent (parity
    UNPINNED): the symmetric Toeplitz ``C[i, j] = N_p((p+1)/2 + i - j)`` of the centred
    cardinal B-spline sampled at the integers (p=3: [1, 4, 1]/6; p=1: identity)."""
    i = np.arange(int(n))
    return cardinal_bspline(int(p), (p + 1) / 2.0 + i[:, None] - i[None, :])


def array_to_mat_stencil(n: int, p: int, C: np.ndarray):
    """`sources/utils.py:104-133`: the entries of C within the 2p+1 band as a 1D
    stencil matrix (host band rows)."""
    from .stencil import StencilMatrix1D
    return StencilMatrix1D(n, p, dense_to_band(np.asarray(C, dtype=np.float64), p))

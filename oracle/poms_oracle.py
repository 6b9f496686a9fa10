"""CPU ORACLE -- test infrastructure only, never part of the product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  It restates the
reference algorithm of the hot path in NumPy/SciPy on global arrays (no
padding tricks, no sum factorisation of the test operator), each function
citing the reference line it follows.

Pinning: ``tests/test_oracle_golden.py`` checks these functions against the
golden vectors generated from the reference itself (``tests/golden/make_golden.py``
imports `pyccel/pyccel_functions.py`, `sources/solvers.py`,
`sources/matrix_assembler.py`, `sources/multilevels.py`, `sources/utils.py`
and runs `sources/mg_jac.py` in this container).  The spl library the
reference delegates to is absent (`requirements.txt:4`, unpinned); where a
result depends only on spl (`matrix_multi_stages`) parity is pinned by
properties instead.
"""
from __future__ import annotations

from math import sqrt

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import splu

__all__ = [
    "band_dense", "band_csr", "kron_dot_pyccel_2d", "kron_product_apply", "kron_sum_apply",
    "kron_sum_csr", "kron_sum_diag", "residual", "damped_jacobi", "jacobi", "pcg",
    "vcycle_two_level", "knots_to_insert", "to_bnd", "gbtrf", "gbtrs", "kron_solve", "pcg_glt", "crl",
    "cardinal_bspline", "collocation_cardinal_splines", "assembly_varcoef",
]


# ---------------------------------------------------------------------------
# 1D band helpers (spl 1D StencilMatrix: M[i, k] = a(i, i+k-p))
# ---------------------------------------------------------------------------
def band_dense(band: np.ndarray) -> np.ndarray:
    n, w = band.shape
    p = (w - 1) // 2
    A = np.zeros((n, n))
    for k in range(w):
        off = k - p
        i = np.arange(max(0, -off), min(n, n - off))
        A[i, i + off] = band[i, k]
    return A


def band_csr(band: np.ndarray) -> sp.csr_matrix:
    return sp.csr_matrix(band_dense(band))


# ---------------------------------------------------------------------------
# pyccel/pyccel_functions.py:4-21 -- the native Kron kernel, loop semantics
# ---------------------------------------------------------------------------
def kron_dot_pyccel_2d(starts, ends, pads, X, X_tmp, Y, A, B):
    """Restatement of `kron_dot_pyccel_2d` (`pyccel/pyccel_functions.py:4-21`).

    Pass 1 (:12-15) runs over the first-axis rows INCLUDING ghosts
    ``j1 in [s1-p1, e1+p1]`` and the owned columns; pass 2 (:17-19) over owned
    rows.  Vectorised over the owned column range, loops kept over rows/taps.
    """
    s1, s2 = int(starts[0]), int(starts[1])
    e1, e2 = int(ends[0]), int(ends[1])
    p1, p2 = int(pads[0]), int(pads[1])
    cols = np.arange(s2, e2 + 1)
    lc = cols - s2 + p2                         # local padded column of i2
    for j1 in range(s1 - p1, e1 + p1 + 1):      # :12
        acc = np.zeros(len(cols))
        for k in range(2 * p2 + 1):             # :15 sum over k
            acc += X[j1 + p1 - s1, cols - s2 + k] * B[cols, k]
        X_tmp[j1 + p1 - s1, lc] = acc
    for i1 in range(s1, e1 + 1):                # :17
        acc = np.zeros(len(cols))
        for k in range(2 * p1 + 1):             # :19
            acc += A[i1, k] * X_tmp[i1 - s1 + k, lc]
        Y[i1 - s1 + p1, lc] = acc
    return Y


# ---------------------------------------------------------------------------
# Operators on global (unpadded) arrays, zero ghosts (non-periodic)
# ---------------------------------------------------------------------------
def _axis_apply(F: sp.csr_matrix, X: np.ndarray, axis: int) -> np.ndarray:
    Xm = np.moveaxis(X, axis, 0)
    sh = Xm.shape
    Y = F @ Xm.reshape(sh[0], -1)
    return np.moveaxis(np.asarray(Y).reshape((F.shape[0],) + sh[1:]), 0, axis)


def kron_product_apply(X: np.ndarray, F: list) -> np.ndarray:
    """(F0 ⊗ F1 ⊗ ...) vec(X), C order (`utils.kron_dot_ref`, `sources/utils.py:43-62`)."""
    Y = X
    for d, f in enumerate(F):
        Y = _axis_apply(band_csr(f) if not sp.issparse(f) else f, Y, d)
    return Y


def kron_sum_apply(X: np.ndarray, M: list, K: list, c: float = 1.0) -> np.ndarray:
    """``c ⊗M + Σ_d (K on axis d, M elsewhere)`` applied term by term.

    This is the operator the reference assembles for ``-Δu + u``
    (`sources/matrix_assembler.py:173`: ``bi0*bj0 + bix*bjx + biy*bjy``), one
    Kronecker term at a time (no shared partial products, unlike the kernel).
    """
    nd = X.ndim
    Mc = [band_csr(m) for m in M]
    Kc = [band_csr(k) for k in K]
    Y = c * kron_product_apply(X, Mc)
    for d in range(nd):
        Y = Y + kron_product_apply(X, [Kc[e] if e == d else Mc[e] for e in range(nd)])
    return Y


def kron_sum_csr(M: list, K: list, c: float = 1.0) -> sp.csr_matrix:
    nd = len(M)
    Mc = [band_csr(m) for m in M]
    Kc = [band_csr(k) for k in K]

    def kr(ms):
        out = ms[0]
        for m in ms[1:]:
            out = sp.kron(out, m, format="csr")
        return out

    A = c * kr(Mc)
    for d in range(nd):
        A = A + kr([Kc[e] if e == d else Mc[e] for e in range(nd)])
    return A.tocsr()


def kron_sum_diag(M: list, K: list, c: float = 1.0) -> np.ndarray:
    nd = len(M)
    dM = [m[:, (m.shape[1] - 1) // 2] for m in M]
    dK = [k[:, (k.shape[1] - 1) // 2] for k in K]

    def outer(vs):
        out = vs[0]
        for v in vs[1:]:
            out = np.multiply.outer(out, v)
        return out

    D = c * outer(dM)
    for d in range(nd):
        D = D + outer([dK[e] if e == d else dM[e] for e in range(nd)])
    return D


def residual(apply, b, x):
    """``r = b - A.dot(x)`` (`sources/solvers.py:85`)."""
    return b - apply(x)


# ---------------------------------------------------------------------------
# sources/solvers.py restated on NumPy arrays
# ---------------------------------------------------------------------------
def jacobi(diag, b):
    """`sources/solvers.py:139-163`: x = b / diag(A)."""
    return b / diag


def damped_jacobi(apply, diag, b, x0=None, tol=1e-6, maxiter=10, return_info=False):
    """`sources/solvers.py:167-235` (omega = 2/3, break after the update)."""
    omega = 2.0 / 3
    x = 0.0 * b.copy() if x0 is None else x0.copy()
    tol_sqr = tol ** 2
    k, nrmr = 0, 0.0
    for k in range(1, maxiter + 1):
        r = b - apply(x)                # :209
        dr = omega * r / diag           # :211-213
        x = x + dr                      # :217
        nrmr = float(np.vdot(dr, dr))   # :219
        if nrmr < tol_sqr:
            k -= 1
            break
    if return_info:
        return x, {"niter": k, "success": nrmr < tol_sqr, "res_norm": sqrt(nrmr)}
    return x


def crl(apply, b, x0=None, tol=1e-5, maxiter=1000):
    """`sources/solvers.py:3-65` (conjugate residual; stop test ``s.r < tol**2``, :38)."""
    x = 0.0 * b.copy() if x0 is None else x0.copy()
    r = b - apply(x)
    p = r.copy()
    q = apply(p)
    s = q.copy()
    sr = float(np.vdot(s, r))
    tol_sqr = tol ** 2
    k = 0
    for k in range(1, maxiter + 1):
        if sr < tol_sqr:
            k -= 1
            break
        alpha = sr / float(np.vdot(q, q))
        x = x + alpha * p
        r = r - alpha * q
        s = apply(r)
        srold = sr
        sr = float(np.vdot(s, r))
        beta = sr / srold
        p = r + beta * p
        q = s + beta * q
    return x, {"niter": k, "success": sr < tol_sqr, "res_norm": sqrt(sr)}


def pcg(apply, psolve, b, x0=None, tol=1e-6, maxiter=100):
    """`sources/solvers.py:69-135` (stop test ``r.r < tol*||r0||``, :113)."""
    x = 0.0 * b.copy() if x0 is None else x0.copy()
    r = b - apply(x)
    nrmr0 = sqrt(float(np.vdot(r, r)))
    s = psolve(r)
    p = s
    sr = float(np.vdot(s, r))
    k, nrmr = 0, nrmr0 * nrmr0
    for k in range(1, maxiter + 1):
        q = apply(p)
        alpha = sr / float(np.vdot(p, q))
        x = x + alpha * p
        r = r - alpha * q
        nrmr = float(np.vdot(r, r))
        if nrmr < tol * nrmr0:
            k -= 1
            break
        s = psolve(r)
        srold = sr
        sr = float(np.vdot(s, r))
        beta = sr / srold
        p = s + beta * p
    return x, {"niter": k, "success": nrmr < tol * nrmr0, "res_norm": sqrt(nrmr)}


# ---------------------------------------------------------------------------
# Kronecker direct solve (GLT preconditioner): sources/kron_product.py:93-238,
# pyccel/pyccel_functions.py:26-248.  LAPACK band storage, dgbtf2 / dgbtrs.
# ---------------------------------------------------------------------------
def to_bnd(A: np.ndarray):
    """`sources/kron_product.py:179-191`: ``A_bnd[la+ua+i-j, j] = A[i, j]`` with ``la``
    spare rows for fill-in."""
    A = np.asarray(A, dtype=np.float64)
    ii, jj = np.nonzero(A)
    la = int(max(0, (ii - jj).max())) if ii.size else 0
    ua = int(max(0, (jj - ii).max())) if ii.size else 0
    ab = np.zeros((1 + ua + 2 * la, A.shape[0]), order="F")
    ab[la + ua + ii - jj, jj] = A[ii, jj]
    return ab, la, ua


def gbtrf(ab: np.ndarray, kl: int, ku: int):
    """LAPACK dgbtf2 (partial pivoting, the path scipy's dgbtrf takes for kl < 32),
    0-based: returns (factorised copy, ipiv, info).  Pure-Python loops: small n."""
    ab = np.array(ab, dtype=np.float64, order="F", copy=True)
    n = ab.shape[1]
    kv = kl + ku
    for j in range(ku + 1, min(kv, n)):
        ab[kv - j:kl, j] = 0.0
    ipiv = np.zeros(n, dtype=np.int64)
    ju, info = 0, 0
    for j in range(n):
        if j + kv < n:
            ab[:kl, j + kv] = 0.0
        km = min(kl, n - 1 - j)
        jp = int(np.argmax(np.abs(ab[kv:kv + km + 1, j])))   # first maximum (idamax)
        ipiv[j] = j + jp
        if ab[kv + jp, j] != 0.0:
            ju = max(ju, min(j + ku + jp, n - 1))
            if jp != 0:
                for c in range(ju - j + 1):
                    ab[kv + jp - c, j + c], ab[kv - c, j + c] = ab[kv - c, j + c], ab[kv + jp - c, j + c]
            if km > 0:
                ab[kv + 1:kv + km + 1, j] *= 1.0 / ab[kv, j]
                for k in range(1, ju - j + 1):
                    y = ab[kv - k, j + k]
                    if y != 0.0:
                        ab[kv + 1 - k:kv + km + 1 - k, j + k] -= ab[kv + 1:kv + km + 1, j] * y
        elif info == 0:
            info = j + 1
    return ab, ipiv, info


def gbtrs(ab: np.ndarray, kl: int, ku: int, ipiv: np.ndarray, b: np.ndarray) -> np.ndarray:
    """LAPACK dgbtrs (no transpose) on the leading axis of ``b`` (any trailing shape)."""
    x = np.array(b, dtype=np.float64, copy=True)
    n = ab.shape[1]
    kd = kl + ku
    for j in range(n - 1):
        lm = min(kl, n - 1 - j)
        l = int(ipiv[j])
        if l != j:
            x[[l, j]] = x[[j, l]]
        if lm:
            x[j + 1:j + 1 + lm] -= np.multiply.outer(ab[kd + 1:kd + 1 + lm, j], x[j])
    for j in range(n - 1, -1, -1):        # dtbsv, upper, column form
        x[j] = x[j] / ab[kd, j]
        i0 = max(0, j - kd)
        if j > i0:
            x[i0:j] -= np.multiply.outer(ab[kd - (j - i0):kd, j], x[j])
    return x


def kron_solve(F: list, Y: np.ndarray) -> np.ndarray:
    """``X = (F0^-1 ⊗ F1^-1 [⊗ F2^-1]) Y`` on a global interior array, axis 0 first
    (`pyccel/pyccel_functions.py:150-171,216-246`)."""
    X = np.array(Y, dtype=np.float64, copy=True)
    for d, Fd in enumerate(F):
        ab, kl, ku = to_bnd(Fd)
        lu, ipiv, info = gbtrf(ab, kl, ku)
        if info:
            raise np.linalg.LinAlgError(f"factor {d} is singular (info {info})")
        X = np.moveaxis(gbtrs(lu, kl, ku, ipiv, np.moveaxis(X, d, 0)), 0, d)
    return X


def pcg_glt(apply, F: list, b, x0=None, tol=1e-6, maxiter=100):
    """`sources/solvers.py:239-306`: pcg with ``psolve = kron_solve_par(M2, M1, .)``
    (here ``F[d]`` acts on axis ``d``; the reference passes ``(M2, M1)``)."""
    shape = tuple(np.asarray(f).shape[0] for f in F)
    return pcg(apply, lambda r: kron_solve(F, r.reshape(shape)).reshape(r.shape), b, x0=x0, tol=tol,
               maxiter=maxiter)


def cardinal_bspline(p: int, x):
    """Cardinal B-spline of degree p on the knots 0, 1, ..., p+1 (truncated-power form)."""
    from math import comb, factorial
    x = np.asarray(x, dtype=np.float64)
    s = np.zeros_like(x)
    for k in range(p + 2):
        s += (-1) ** k * comb(p + 1, k) * np.where(x > k, (x - k) ** p, 0.0)
    return np.where((x > 0) & (x < p + 1), s / factorial(p), 0.0)


def collocation_cardinal_splines(p: int, n: int) -> np.ndarray:
    """spl's ``collocation_cardinal_splines(p, n)`` (spl absent, restated, UNPINNED):
    the n x n symmetric Toeplitz matrix ``C[i, j] = N_p((p+1)/2 + i - j)`` of the centred
    cardinal B-spline sampled at the integers."""
    i = np.arange(n)
    return cardinal_bspline(p, (p + 1) / 2.0 + i[:, None] - i[None, :])


# ---------------------------------------------------------------------------
# Quadrature assembly: sources/matrix_assembler.py:84-179 (assembly_2d), in d
# dimensions and with coefficient fields a, c at the quadrature points
# ---------------------------------------------------------------------------
def assembly_varcoef(knots, p, a=None, c=None, mass_coef=1.0):
    """spl-layout stencil ``_data`` of ``-div(a grad u) + c u``: element loop, local
    basis pairs, quadrature sum per element added into ``M[i, j - i]`` as
    `sources/matrix_assembler.py:136-177` (a = c = 1 there).  Basis tables from the
    spl stand-in's ``SplineSpace`` (its own Cox-de Boor evaluation).  ``a``/``c``:
    arrays over the global quadrature grid ``(nel_0 nq_0, nel_1 nq_1, ...)`` or None."""
    from itertools import product
    from oracle.spl_standin import SplineSpace
    S = [SplineSpace(pd, knots=np.asarray(T, float)) for T, pd in zip(knots, p)]
    nd = len(S)
    n = [s.nbasis for s in S]
    nq = [s.quad_order for s in S]
    out = np.zeros(tuple(ni + 2 * pi for ni, pi in zip(n, p)) + tuple(2 * pi + 1 for pi in p))
    for es in np.ndindex(*[s.ne for s in S]):
        first = [int(S[d].spans[es[d]]) - p[d] - 1 for d in range(nd)]
        B = [S[d].basis[:, :, :, es[d]] for d in range(nd)]          # (p+1, 2, nq)
        w = S[0].weights[:, es[0]]
        for d in range(1, nd):
            w = np.multiply.outer(w, S[d].weights[:, es[d]])
        blk = tuple(slice(es[d] * nq[d], (es[d] + 1) * nq[d]) for d in range(nd))
        ca = 1.0 if a is None else a[blk]
        cc = mass_coef if c is None else c[blk]

        def tens(il, der_axis):
            t = B[0][il[0], 1 if der_axis == 0 else 0]
            for d in range(1, nd):
                t = np.multiply.outer(t, B[d][il[d], 1 if der_axis == d else 0])
            return t

        for il in product(*[range(pd + 1) for pd in p]):
            bi = [tens(il, -1)] + [tens(il, d) for d in range(nd)]
            for jl in product(*[range(pd + 1) for pd in p]):
                bj = [tens(jl, -1)] + [tens(jl, d) for d in range(nd)]
                grad = bi[1] * bj[1]
                for d in range(2, nd + 1):
                    grad = grad + bi[d] * bj[d]
                v = float(np.sum((cc * bi[0] * bj[0] + ca * grad) * w))
                i = [first[d] + il[d] for d in range(nd)]
                j = [first[d] + jl[d] for d in range(nd)]
                out[tuple(i[d] + p[d] for d in range(nd)) + tuple(j[d] - i[d] + p[d] for d in range(nd))] += v
    return out


# ---------------------------------------------------------------------------
# sources/multilevels.py:7-33 and the mg_jac.py V-cycle
# ---------------------------------------------------------------------------
def knots_to_insert(Tf, nf, pf, Tc, nc, pc):
    """Interior knots ``Tf[pf+1:nf]`` absent (exact equality) from ``Tc[pc+1:nc+1]``.

    The reference scans ``Tc`` from ``pc+1`` until the first larger knot or
    ``j > nc`` (`sources/multilevels.py:17-29`); on a sorted ``Tc`` that is
    membership in ``Tc[pc+1 .. nc]``.
    """
    coarse = set(float(t) for t in Tc[pc + 1:nc + 1])
    return np.array([t for t in Tf[pf + 1:nf] if float(t) not in coarse], dtype=np.float64)


def vcycle_two_level(M, K, P1, b, c=1.0, tol=1e-6, maxiter=10, x0=None, reorder=False, glt=None):
    """`sources/mg_jac.py:84-119` on global arrays with materialised R, P, Ac, splu.

    ``glt`` (list of per-axis 1D matrices): the post-smoother is instead
    `sources/mg_glt.py:113-123`, ``pcg_glt`` with ``maxiter = p + 1``, whose
    preconditioner solves with ``glt[d]`` on axis ``d``.

    ``reorder=True`` applies the fine operator term by term instead of through
    the assembled CSR matrix: same arithmetic, different summation order (used
    to measure how much the reference algorithm amplifies roundoff).
    """
    nd = b.ndim
    A = kron_sum_csr(M, K, c)
    D = kron_sum_diag(M, K, c).reshape(-1)
    if reorder:
        apply = lambda v: kron_sum_apply(v.reshape(b.shape), M, K, c).reshape(-1)
    else:
        apply = lambda v: A @ v
    psolve = lambda r: damped_jacobi(apply, D, r)
    bf = b.reshape(-1)
    xf, info_pre = pcg(apply, psolve, bf, x0=None if x0 is None else x0.reshape(-1), tol=tol, maxiter=maxiter)
    Pm = sp.csr_matrix(P1)
    P = Pm
    for _ in range(nd - 1):
        P = sp.kron(P, Pm, format="csr")
    R = P.T.tocsr()
    Ac = (R @ A @ P).tocsc()
    rf = bf - apply(xf)
    rc = R @ rf
    xc = splu(Ac).solve(rc)
    xf = xf + P @ xc
    if glt is not None:
        p = (M[0].shape[1] - 1) // 2
        xf2, info_pos = pcg_glt(apply, glt, bf, x0=xf, tol=tol, maxiter=p + 1)
    else:
        xf2, info_pos = pcg(apply, psolve, bf, x0=xf, tol=tol, maxiter=maxiter)
    return xf2.reshape(b.shape), info_pre, info_pos


def vcycle_multilevel(Ms, Ks, P1s, b, c=1.0, tol=1e-6, maxiters=None, x0=None, reorder=False):
    """Recursive V-cycle over L levels (the reference's
    two-level cycle `sources/mg_jac.py:84-119` applied at every level).

    Level 0 is the finest.  ``Ms[l]``, ``Ks[l]``: per-axis band factors of level
    l (used on level 0 only: coarser operators are the materialised Galerkin
    products R A P, as in the reference); ``P1s[l]``: 1D prolongation from level
    l+1 to level l.  ``maxiters[l]``: pcg iterations of the pre / post smoothing
    on level l (default 10, the reference's).  The coarsest level is solved with
    ``splu``.  Returns ``(x, infos)`` with ``infos[l] = (info_pre, info_post)``
    of the first visit of level l.
    """
    L = len(P1s) + 1
    nd = b.ndim
    maxiters = [10] * (L - 1) if maxiters is None else list(maxiters)
    A0 = kron_sum_csr(Ms[0], Ks[0], c)
    As, Ps = [A0], []
    for l in range(L - 1):
        Pm = sp.csr_matrix(P1s[l])
        P = Pm
        for _ in range(nd - 1):
            P = sp.kron(P, Pm, format="csr")
        Ps.append(P)
        As.append((P.T @ As[l] @ P).tocsr())
    infos = [None] * (L - 1)

    def cycle(l, bl, xl0):
        if l == L - 1:
            return splu(As[l].tocsc()).solve(bl)
        A = As[l]
        D = A.diagonal().copy()
        if l == 0 and reorder:
            apply = lambda v: kron_sum_apply(v.reshape(b.shape), Ms[0], Ks[0], c).reshape(-1)
        else:
            apply = lambda v: A @ v
        psolve = lambda r: damped_jacobi(apply, D, r)
        x, ipre = pcg(apply, psolve, bl, x0=xl0, tol=tol, maxiter=maxiters[l])
        rc = Ps[l].T @ (bl - apply(x))
        ec = cycle(l + 1, rc, None)
        x = x + Ps[l] @ ec
        x, ipos = pcg(apply, psolve, bl, x0=x, tol=tol, maxiter=maxiters[l])
        if infos[l] is None:
            infos[l] = (ipre, ipos)
        return x

    x = cycle(0, b.reshape(-1), None if x0 is None else x0.reshape(-1))
    return x.reshape(b.shape), infos

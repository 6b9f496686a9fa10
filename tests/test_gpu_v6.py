"""v6 (csrc/kron_v6.hip, variant 11): the Kron apply with three columns per lane.

192-lane-column tiles (176 output columns each on the line-aligned layout), so
rows of more than 176 columns have interior tiles (the Toeplitz fast path on
axis 2) beside boundary tiles (the per-lane-column LDS table); waves whose row
lies outside the axis-1 Toeplitz interior take the scalar-coefficient path.
Checked against the oracle (1e-13) and against the general kernel (variant 0)
on the same operator, for p = 1, 2, 3, equal and different axis-1 / axis-2
knot vectors (the SAME12 builds and the others), ragged last tiles in both
directions, and a layout v6 does not take (unaligned: the launch falls back to
v5 and still matches).
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, uniform_knots

pytestmark = pytest.mark.gpu

TOL = 1e-13


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _truncate(F, n0, p):
    G = np.array(F[:n0], copy=True)
    for i in range(n0):
        for k in range(2 * p + 1):
            if not 0 <= i + k - p < n0:
                G[i, k] = 0.0
    return G


@pytest.mark.parametrize("p,n0,N1,N2", [
    (3, 40, 250, 250),    # SAME12, two column tiles (176 + 77)
    (3, 37, 61, 400),     # three column tiles, different axis-1 / axis-2 rows
    (3, 20, 33, 170),     # one column tile: every tile is a boundary tile
    (2, 35, 100, 360),
    (1, 30, 47, 353),
])
def test_v6_apply(gpu, p, n0, N1, N2):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    M1, K1 = assemble_1d(uniform_knots(p, N1), p)
    M2, K2 = assemble_1d(uniform_knots(p, N2), p)
    n1, n2 = N1 + p, N2 + p
    M0, K0 = _truncate(M1, n0, p), _truncate(K1, n0, p)
    Ms, Ks = [M0, M1, M2], [K0, K1, K2]
    npts = (n0, n1, n2)
    V = StencilVectorSpace(npts, [p] * 3, align=True)
    A = KronOperator.laplace(V, Ms, Ks)
    A.set_variant(11)
    assert A.kernel_variant("apply") == 11
    assert A.kernel_variant("jacobi") == 10   # v6 builds only the apply
    rng = np.random.default_rng(n0 + n2)
    x = rng.uniform(-1, 1, npts)
    xv = V.zeros().from_numpy(x)
    y_ref = orc.kron_sum_apply(x, Ms, Ks)
    yv = V.zeros()
    A.dot(xv, out=yv)
    y = yv.to_local_numpy()
    assert rel(y, y_ref) <= TOL
    # ghosts stay zero (v6 stores output columns only)
    full = yv._data.cpu().numpy()
    assert np.count_nonzero(full) == np.count_nonzero(y)
    A.set_variant(0)
    y0 = A.dot(xv).to_local_numpy()
    assert rel(y, y0) <= TOL
    # the slab schedule's launches: interior planes, then both p-plane boundaries in
    # one launch of two plane ranges -- bitwise the single launch
    from poms_amd import _lib, runtime as rt
    A.set_variant(11)
    y2 = V.zeros()
    st = rt.stream_handle()
    _lib.call("poms_op_run_reduce2", A._h, 0, 0.0, rt.ptr(xv._data), rt.ptr(y2._data), None,
              p, n0 - p, 0, 0, None, None, 0, st)
    _lib.call("poms_op_run_reduce2", A._h, 0, 0.0, rt.ptr(xv._data), rt.ptr(y2._data), None,
              0, p, n0 - p, n0, None, None, 0, st)
    np.testing.assert_array_equal(y2.to_local_numpy(), y)


def test_v6_unaligned_falls_back(gpu):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, 200
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    npts = (24, n, n)
    Ms, Ks = [_truncate(M, 24, p), M, M], [_truncate(K, 24, p), K, K]
    V = StencilVectorSpace(npts, [p] * 3, align=False)
    A = KronOperator.laplace(V, Ms, Ks)
    A.set_variant(11)
    x = np.random.default_rng(5).uniform(-1, 1, npts)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert rel(y, orc.kron_sum_apply(x, Ms, Ks)) <= TOL

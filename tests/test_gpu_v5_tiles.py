"""v5 (csrc/kron_v5.hip) at p = 3 where the headline grid takes it: axes 1 and 2
share their Toeplitz rows (equal cell counts: the SAME12 builds, and the
16-wave two-sweeps-from-zero build), several 112/120-column tiles so that whole
tiles lie inside the axis-2 interior (the constant-row fast path) beside the
boundary tiles (per-column LDS tables), on the line-aligned layout (halo lanes
not fetched) and the unaligned one.  The generic kernel cases
(tests/test_gpu_kernels.py) never reach the fast path: their n2 fits one tile.

Axis 0 is the first n0 rows of the same 1D factors (zero past column n0), so its
middle rows are the axis-1 Toeplitz row and its first and last p are not.
Every epilogue is checked against the oracle (1e-13), and v5 against the general
kernel (variant 0) on the same operator.
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


@pytest.mark.parametrize("n0,N,align", [(60, 250, True), (33, 240, False), (90, 250, True)])
def test_v5_interior_tiles_epilogues(gpu, n0, N, align):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    M0, K0 = _truncate(M, n0, p), _truncate(K, n0, p)
    Ms, Ks = [M0, M, M], [K0, K, K]
    npts = (n0, n, n)
    V = StencilVectorSpace(npts, [p] * 3, align=align)
    A = KronOperator.laplace(V, Ms, Ks)
    A.set_variant(8)
    assert A.kernel_variant("jacobi") == 10 and A.kernel_variant("apply") == 10
    rng = np.random.default_rng(n0)
    x = rng.uniform(-1, 1, npts)
    b = rng.uniform(-1, 1, npts)
    xv, bv = V.zeros().from_numpy(x), V.zeros().from_numpy(b)
    y_ref = orc.kron_sum_apply(x, Ms, Ks)
    D = orc.kron_sum_diag(Ms, Ks)
    w = 2.0 / 3.0
    y = A.dot(xv).to_local_numpy()
    assert rel(y, y_ref) <= TOL
    r = A.residual(bv, xv).to_local_numpy()
    assert rel(r, b - y_ref) <= TOL
    xo = V.empty()
    nrm = A.jacobi_sweep(bv, xv, xo, w, want_norm=True)
    dr = w * (b - y_ref) / D
    assert rel(xo.to_local_numpy(), x + dr) <= TOL
    assert abs(nrm - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr))
    # the general kernel on the same operator
    outs = {}
    for v in (10, 0):
        A.set_variant(v)
        xo2 = V.empty()
        A.jacobi_sweep(bv, xv, xo2, w)
        outs[v] = (A.dot(xv).to_local_numpy(), xo2.to_local_numpy())
    assert rel(outs[10][0], outs[0][0]) <= TOL and rel(outs[10][1], outs[0][1]) <= TOL
    # two sweeps from zero and apply + dot
    A.set_variant(8)
    y0 = V.zeros()
    A.jacobi_from_zero(bv, y0, w)
    x1 = w * b / D
    x2 = x1 + w * (b - orc.kron_sum_apply(x1, Ms, Ks)) / D
    assert rel(y0.to_local_numpy(), x2) <= TOL

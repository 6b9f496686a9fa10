"""m2 (csrc/kron_m2.hip, variant 12): the 2D row-marching kernel, against the oracle.

Every epilogue the 2D V-cycle uses (apply, residual, damped-Jacobi sweep with its
norm and the fused x_out . b, apply + x . Ax) at p = 1, 2, 3 on the line-aligned
layout (the V-cycle's), spline and random band factors, widths that fill the last
112-column tile partly or exactly, and row chunks from 1 row to more than the grid;
a block with data in its ghosts (a 2D spl Cart block, p = 2); and the fall-back to
the round-4 kernels where rows are not 16-B aligned.  Tolerances as in
test_gpu_kernels.py: 1e-13 normwise, sums 1e-12 relative.
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, uniform_knots

pytestmark = pytest.mark.gpu

TOL = 1e-13


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _factors(p, N, rng, kind):
    if kind == "spline":
        return assemble_1d(uniform_knots(p, N), p)
    n = N + p
    M = rng.uniform(-1, 1, (n, 2 * p + 1))
    K = rng.uniform(-1, 1, (n, 2 * p + 1))
    for B in (M, K):
        for i in range(n):
            for k in range(2 * p + 1):
                if not 0 <= i + k - p < n:
                    B[i, k] = 0.0
    M[:, p] += 4.0
    K[:, p] = np.abs(K[:, p]) + 1.0
    return M, K


@pytest.mark.parametrize("p,cells", [(1, (37, 70)), (2, (33, 129)), (3, (64, 64)), (3, (61, 221)), (3, (200, 109))])
@pytest.mark.parametrize("kind", ["spline", "random"])
@pytest.mark.parametrize("chunk", [0, 1, 5, 300])
def test_m2_epilogues_match_oracle(gpu, p, cells, kind, chunk):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    rng = np.random.default_rng(100 * p + cells[1] + len(kind))
    M, K = zip(*[_factors(p, N, rng, kind) for N in cells])
    npts = tuple(N + p for N in cells)
    V = StencilVectorSpace(npts, (p, p), align=True)
    c = 1.0 if kind == "spline" else 0.7
    A = KronOperator.laplace(V, M, K, mass_coef=c)
    A.set_chunk(chunk)
    x = rng.uniform(-1, 1, npts)
    b = rng.uniform(-1, 1, npts)
    y_ref = orc.kron_sum_apply(x, M, K, c)
    xv, bv = V.zeros().from_numpy(x), V.zeros().from_numpy(b)
    y = A.dot(xv).to_local_numpy()
    assert A.last_variant == 12, "m2 did not run"
    assert rel(y, y_ref) <= TOL
    r = A.residual(bv, xv).to_local_numpy()
    assert A.last_variant == 12
    assert rel(r, b - y_ref) <= TOL
    D = orc.kron_sum_diag(M, K, c)
    dr = (2.0 / 3.0) * (b - y_ref) / D
    xo = V.empty()
    nrm = A.jacobi_sweep(bv, xv, xo, 2.0 / 3.0, want_norm=True)
    assert A.last_variant == 12
    assert rel(xo.to_local_numpy(), x + dr) <= TOL
    assert abs(nrm - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr))
    nrm2, dot = A.jacobi_sweep(bv, xv, xo, 2.0 / 3.0, want_norm=True, want_dot=True)
    assert abs(nrm2 - nrm) <= 1e-13 * nrm
    assert abs(dot - float(np.vdot(x + dr, b))) <= 1e-12 * abs(float(np.vdot(x + dr, b)))
    ip = A.dot_inner(xv, V.empty())
    assert abs(ip - float(np.vdot(x, y_ref))) <= 1e-12 * abs(float(np.vdot(x, y_ref)))
    # ghosts (and dead pitch columns) stay zero after every launch
    for vec in (xo,):
        data = vec._data.cpu().numpy()
        inner = V.interior(vec._data).cpu().numpy()
        assert np.abs(data).sum() == pytest.approx(np.abs(inner).sum())


@pytest.mark.parametrize("chunk", [0, 3])
def test_m2_chunking_is_bitwise_invariant(gpu, chunk):
    """Row chunks recompute their 2p halo rows with the same arithmetic: results equal
    the one-chunk launch bit for bit."""
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, cells = 3, (90, 150)
    M, K = zip(*[assemble_1d(uniform_knots(p, N), p) for N in cells])
    npts = tuple(N + p for N in cells)
    V = StencilVectorSpace(npts, (p, p), align=True)
    A = KronOperator.laplace(V, M, K)
    xv = V.zeros().from_numpy(np.random.default_rng(4).uniform(-1, 1, npts))
    A.set_chunk(10 ** 6)
    y1 = A.dot(xv).to_local_numpy()
    A.set_chunk(chunk)
    y2 = A.dot(xv).to_local_numpy()
    assert A.last_variant == 12
    assert np.array_equal(y1, y2)


def test_m2_block_with_ghost_data(gpu):
    """A 2D spl Cart block (p = 2): the owned rows / columns are a window of larger
    global factors and every ghost (edges and corners) holds the neighbours' values."""
    import torch
    from poms_amd import _lib
    from poms_amd.stencil import KronOperator, StencilVectorSpace, _widen
    p = 2
    rng = np.random.default_rng(77)
    cells_g = (60, 300)
    Mg, Kg = zip(*[assemble_1d(uniform_knots(p, N), p) for N in cells_g])
    ng = [N + p for N in cells_g]
    s1, s2 = 13, 37
    nl = (29, 170)
    xg = rng.standard_normal(ng)
    V = StencilVectorSpace(list(nl), [p] * 2, align=True)
    bands = {"A1": Mg[0][s1:s1 + nl[0]] + Kg[0][s1:s1 + nl[0]], "B1": Mg[0][s1:s1 + nl[0]],
             "M2": Mg[1][s2:s2 + nl[1]], "K2": Kg[1][s2:s2 + nl[1]]}
    A = KronOperator(V, "sum", {k: _widen(v, p) for k, v in bands.items()}, p)
    _lib.call("poms_op_set_ghost_corners", A._h, 1)
    x = V.zeros()
    full = np.zeros(V.padded_shape)
    full[:, :nl[1] + 2 * p] = xg[s1 - p:s1 + nl[0] + p, s2 - p:s2 + nl[1] + p]
    x._data.copy_(torch.from_numpy(np.ascontiguousarray(full)))
    y = A.dot(x).to_local_numpy()
    assert A.last_variant == 12
    ref = orc.kron_sum_apply(xg, Mg, Kg)[s1:s1 + nl[0], s2:s2 + nl[1]]
    assert rel(y, ref) <= TOL


def test_m2_falls_back_on_unaligned_rows(gpu):
    """Rows that are not 16-B aligned (the exact spl pitch n + 2p, odd here) run the
    round-4 2D kernels, with the same results."""
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, cells = 3, (40, 64)
    M, K = zip(*[assemble_1d(uniform_knots(p, N), p) for N in cells])
    npts = tuple(N + p for N in cells)
    V = StencilVectorSpace(npts, (p, p))
    A = KronOperator.laplace(V, M, K)
    x = np.random.default_rng(2).uniform(-1, 1, npts)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert A.last_variant in (7, 9)
    assert rel(y, orc.kron_sum_apply(x, M, K)) <= TOL

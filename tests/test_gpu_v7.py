"""v7 (csrc/kron_v7.hip, variant 11): the flat-lane p = 3 apply.

Its arithmetic is v5's in the same order (axis 1 pair sums, axis 2 pair sums on
the Toeplitz tiles and per-column rows on the boundary tiles, the axis-0 scatter),
so on the same operator and input it must equal v5 BITWISE; against the oracle
the usual 1e-13.  The plane widths cover every tile plan: wide tiles only
(224 = 2 x 112), one wide tile plus the remainder in a whole wide tile (211),
narrow last columns of 16, 32, 48 and 80 (227, 131, 40, 515-wide via n0 thin
slabs), and rows that do not divide the tile height.  Axis 0 is the first n0 rows
of the 1D factors (its middle rows Toeplitz, its first / last p not).
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd import _lib
from poms_amd.splines import assemble_1d, uniform_knots

pytestmark = pytest.mark.gpu

# v7 is compiled only with POMS_WITH_V7=1 (experimental, slower than v5); without it
# variant 11 runs v5 (test_v7_absent_runs_v5)
V7_BUILT = bool(_lib.lib.poms_variant_built(11))
needs_v7 = pytest.mark.skipif(not V7_BUILT, reason="v7 not in this build (POMS_WITH_V7=1 builds it)")

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


def _op(n0, N1, N2, align=True):
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    M1, K1 = assemble_1d(uniform_knots(p, N1), p)
    M2, K2 = assemble_1d(uniform_knots(p, N2), p)
    Mb, Kb = (M1, K1) if N1 >= N2 else (M2, K2)
    M0, K0 = _truncate(Mb, n0, p), _truncate(Kb, n0, p)
    Ms, Ks = [M0, M1, M2], [K0, K1, K2]
    npts = (n0, N1 + p, N2 + p)
    V = StencilVectorSpace(npts, [p] * 3, align=align)
    return V, KronOperator.laplace(V, Ms, Ks), Ms, Ks, npts


@needs_v7
@pytest.mark.parametrize("n0,N1,N2", [
    (20, 221, 221),    # 224 x 224: two wide tiles, no narrow column
    (17, 208, 208),    # 211: the remainder (99) takes a whole wide tile
    (12, 224, 224),    # 227: two wide tiles + a 16-column narrow tile
    (13, 128, 128),    # 131: one wide tile + a 32-column narrow tile
    (30, 37, 37),      # 40: no wide tile, one 48-column narrow tile
    (9, 300, 512),     # 303 x 515: four wide tiles + an 80-column narrow tile (the headline width)
    (25, 77, 150),     # distinct axis-1 / axis-2 rows (the two-constant-set build)
])
def test_v7_apply_matches_v5_bitwise_and_oracle(gpu, n0, N1, N2):
    V, A, Ms, Ks, npts = _op(n0, N1, N2)
    A.set_variant(11)
    assert A.kernel_variant("apply") == 11 and A.kernel_variant("jacobi") == 11
    rng = np.random.default_rng(n0 * 7 + N2)
    x = rng.uniform(-1, 1, npts)
    xv = V.zeros().from_numpy(x)
    y7 = A.dot(xv).to_local_numpy()
    assert A.last_variant == 11, "v7 did not run (a per-call fall-back took over)"
    y_ref = orc.kron_sum_apply(x, Ms, Ks)
    assert rel(y7, y_ref) <= TOL
    A.set_variant(10)
    y5 = A.dot(xv).to_local_numpy()
    assert np.array_equal(y7, y5), f"v7 != v5 at {int((y7 != y5).sum())} points"
    # ghosts and dead pitch columns stay zero
    A.set_variant(11)
    yv = V.zeros()   # (A.dot(x) allocates with torch.empty: the buffer's alignment slack is not zeroed)
    A.dot(xv, out=yv)
    rest = yv._store.clone()   # the whole buffer (ghosts, dead pitch columns) minus the interior
    V.interior(V.view(rest)).zero_()
    assert not bool(rest.any())


@needs_v7
@pytest.mark.parametrize("n0,N1,N2", [(20, 221, 221), (12, 224, 224), (9, 300, 512), (25, 77, 150), (30, 37, 37)])
def test_v7_epilogues_match_v5(gpu, n0, N1, N2):
    """Residual, Jacobi sweep (norm, and the fused x_out . b), apply + x.Ax: the
    vectors equal v5's bitwise; the per-block sums are added in another block order,
    so the scalars agree to 1e-13 (and with the oracle)."""
    V, A, Ms, Ks, npts = _op(n0, N1, N2)
    rng = np.random.default_rng(n0 + 3 * N2)
    x, b = rng.uniform(-1, 1, npts), rng.uniform(-1, 1, npts)
    xv, bv = V.zeros().from_numpy(x), V.zeros().from_numpy(b)
    w = 2.0 / 3.0
    out = {}
    for v in (11, 10):
        A.set_variant(v)
        r = V.zeros()
        A.residual(bv, xv, out=r)
        assert A.last_variant == v
        xo1, xo2 = V.zeros(), V.zeros()
        n1 = A.jacobi_sweep(bv, xv, xo1, w, want_norm=True)
        assert A.last_variant == v
        n2, d2 = A.jacobi_sweep(bv, xv, xo2, w, want_norm=True, want_dot=True)
        y = V.zeros()
        xy = A.dot_inner(xv, y)
        assert A.last_variant == v
        out[v] = (r.to_local_numpy(), xo1.to_local_numpy(), xo2.to_local_numpy(), y.to_local_numpy(), n1, n2, d2, xy)
    for i in range(4):
        assert np.array_equal(out[11][i], out[10][i]), f"vector {i}: {int((out[11][i] != out[10][i]).sum())} points differ"
    for i in range(4, 8):
        assert abs(out[11][i] - out[10][i]) <= 1e-13 * abs(out[10][i]), (i, out[11][i], out[10][i])
    y_ref = orc.kron_sum_apply(x, Ms, Ks)
    D = orc.kron_sum_diag(Ms, Ks).reshape(npts)
    dr = w * (b - y_ref) / D
    assert rel(out[11][0], b - y_ref) <= TOL and rel(out[11][1], x + dr) <= TOL
    assert abs(out[11][4] - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr))
    assert abs(out[11][6] - float(np.vdot(x + dr, b))) <= 1e-12 * abs(float(np.vdot(x + dr, b)))
    assert abs(out[11][7] - float(np.vdot(x, y_ref))) <= 1e-12 * abs(float(np.vdot(x, y_ref)))


def test_v7_unaligned_layout_falls_back(gpu):
    V, A, Ms, Ks, npts = _op(10, 40, 40, align=False)
    A.set_variant(11)
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, npts)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert A.last_variant == 10
    assert rel(y, orc.kron_sum_apply(x, Ms, Ks)) <= TOL


@needs_v7
def test_v7_headline_grid_matches_v5(gpu):
    """515^3 (the bench grid, 5 tile columns: 4 x 112 + 80): v7 == v5 bitwise on a
    random input, with several axis-0 chunk lengths (chunk boundaries move)."""
    import torch
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, 512
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x, y5, y7 = V.zeros(), V.zeros(), V.zeros()
    g = torch.Generator(device="cuda").manual_seed(5)
    V.interior(x._data).uniform_(-1, 1, generator=g)
    A.set_variant(10)
    A.dot(x, out=y5)
    A.set_variant(11)
    for ch in (0, 37, 200):
        A.set_chunk(ch)
        y7._data.fill_(float("nan"))
        A.dot(x, out=y7)
        assert A.last_variant == 11
        assert bool(torch.equal(V.interior(y7._data), V.interior(y5._data))), f"chunk {ch}"
    A.set_chunk(0)


@pytest.mark.skipif(V7_BUILT, reason="v7 is built")
def test_v7_absent_runs_v5(gpu):
    """Without v7 in the library, asking for variant 11 runs v5 (last_variant 10) with
    v5's results; a v7 diagnostic build asked for by number fails loudly."""
    V, A, _, _, npts = _op(20, 40, 131)
    x = V.zeros().from_numpy(np.random.default_rng(5).uniform(-1, 1, npts))
    y5 = A.dot(x).to_local_numpy()
    A.set_variant(11)
    y = A.dot(x).to_local_numpy()
    assert A.last_variant == 10
    assert np.array_equal(y, y5)
    A.set_variant(121)
    with pytest.raises(_lib.PomsError):
        A.dot(x)

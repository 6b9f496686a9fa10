"""GPU parity of the fused Kronecker kernels against the CPU oracle (fp64).

Tolerances: one operator apply / residual / Jacobi sweep
<= 1e-13 normwise relative; pointwise checks use atol scaled by ||y||_inf
(cancellation gives ~5e-13 pointwise).
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, uniform_knots, make_open_knots

pytestmark = pytest.mark.gpu

TOL = 1e-13


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _factors(p, N, rng=None, kind="spline"):
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
    M[:, p] += 4.0  # keep diag(A) away from zero (Jacobi divides by it)
    K[:, p] = np.abs(K[:, p]) + 1.0
    return M, K


def _space(npts, pads):
    from poms_amd.stencil import StencilVectorSpace
    return StencilVectorSpace(npts, pads)


CASES = [
    # (ndim, cells per axis, p)
    (1, (40,), 2),
    (2, (37, 70), 1), (2, (64, 64), 3), (2, (33, 129), 2), (2, (20, 21), 5), (2, (24, 30), 4),
    (3, (9, 17, 70), 1), (3, (20, 24, 65), 2), (3, (25, 18, 70), 3), (3, (16, 16, 16), 4),
    (3, (14, 12, 66), 5),
]


VARIANTS = [0, 4, 7, 8, 9, 10]


@pytest.mark.parametrize("ndim,cells,p", CASES)
@pytest.mark.parametrize("kind", ["spline", "random"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_apply_residual_jacobi(gpu, ndim, cells, p, kind, variant):
    from poms_amd.stencil import KronOperator
    rng = np.random.default_rng(1000 * ndim + 10 * p + len(kind))
    M, K = zip(*[_factors(p, N, rng, kind) for N in cells])
    npts = tuple(N + p for N in cells)
    V = _space(npts, (p,) * ndim)
    c = 1.0 if kind == "spline" else 0.7
    A = KronOperator.laplace(V, M, K, mass_coef=c)
    if variant and ndim == 1:
        pytest.skip("1D embeds a pad-0 axis: general kernel only")
    A.set_variant(variant)
    x = rng.uniform(-1, 1, npts)
    b = rng.uniform(-1, 1, npts)
    y_ref = orc.kron_sum_apply(x, M, K, c)
    xv = V.zeros().from_numpy(x)
    bv = V.zeros().from_numpy(b)
    y = A.dot(xv).to_local_numpy()
    assert rel(y, y_ref) <= TOL
    assert np.max(np.abs(y - y_ref)) <= 1e-12 * np.max(np.abs(y_ref))
    r = A.residual(bv, xv).to_local_numpy()
    assert rel(r, b - y_ref) <= TOL
    D = orc.kron_sum_diag(M, K, c)
    xo = V.empty()
    nrm = A.jacobi_sweep(bv, xv, xo, 2.0 / 3.0, want_norm=True)
    dr_ref = (2.0 / 3.0) * (b - y_ref) / D
    assert rel(xo.to_local_numpy(), x + dr_ref) <= TOL
    assert abs(nrm - float(np.vdot(dr_ref, dr_ref))) <= 1e-12 * float(np.vdot(dr_ref, dr_ref))
    # ghosts untouched (zero) after every kernel
    for vec in (xo,):
        data = vec._data.cpu().numpy()
        inner = V.interior(vec._data).cpu().numpy()
        assert np.abs(data).sum() == pytest.approx(np.abs(inner).sum())


@pytest.mark.parametrize("ndim,cells,p", [(2, (30, 50), 2), (3, (12, 20, 70), 3), (3, (10, 9, 33), 5)])
@pytest.mark.parametrize("variant", VARIANTS)
def test_product_apply(gpu, ndim, cells, p, variant):
    from poms_amd.stencil import KronOperator
    rng = np.random.default_rng(7 + p)
    npts = tuple(N + p for N in cells)
    F = []
    for n in npts:
        B = rng.uniform(-1, 1, (n, 2 * p + 1))
        for i in range(n):
            for k in range(2 * p + 1):
                if not 0 <= i + k - p < n:
                    B[i, k] = 0.0
        F.append(B)
    V = _space(npts, (p,) * ndim)
    A = KronOperator.product(V, F)
    A.set_variant(variant)
    x = rng.uniform(-1, 1, npts)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert rel(y, orc.kron_product_apply(x, F)) <= TOL


@pytest.mark.parametrize("chunk", [1, 2, 5, 16, 0])
@pytest.mark.parametrize("variant", VARIANTS)
def test_chunking_invariance(gpu, chunk, variant):
    """Output independent of the axis-0 chunking (halo recomputation is exact)."""
    from poms_amd.stencil import KronOperator
    p, cells = 3, (40, 20, 64)
    M, K = zip(*[_factors(p, N) for N in cells])
    npts = tuple(N + p for N in cells)
    V = _space(npts, (p,) * 3)
    A = KronOperator.laplace(V, M, K)
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, npts)
    A.set_chunk(chunk)
    A.set_variant(variant)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert rel(y, orc.kron_sum_apply(x, M, K)) <= TOL


def test_vector_ops(gpu):
    from poms_amd.stencil import KronOperator
    p, cells = 2, (20, 17, 70)
    npts = tuple(N + p for N in cells)
    V = _space(npts, (p,) * 3)
    rng = np.random.default_rng(5)
    a, b = rng.uniform(-1, 1, npts), rng.uniform(-1, 1, npts)
    av, bv = V.zeros().from_numpy(a), V.zeros().from_numpy(b)
    assert abs(av.dot(bv) - float(np.vdot(a, b))) <= 1e-12 * np.sum(np.abs(a * b))
    np.testing.assert_allclose((av + 2.5 * bv).to_local_numpy(), a + 2.5 * b, rtol=0, atol=1e-15)
    np.testing.assert_allclose((av - bv).to_local_numpy(), a - b, rtol=0, atol=1e-15)
    c = av.copy()
    c *= -3.0
    np.testing.assert_allclose(c.to_local_numpy(), -3.0 * a, rtol=0, atol=1e-15)
    assert av[3, 4, 5] == a[3, 4, 5]
    flat = av.toarray()
    np.testing.assert_array_equal(flat, a.reshape(-1))


@pytest.mark.parametrize("ndim,npts,p,align", [(3, (9, 7, 21), 3, True), (3, (9, 7, 21), 2, False),
                                               (2, (13, 40), 3, True), (1, (33,), 2, False)])
def test_zero_ghosts(gpu, ndim, npts, p, align):
    """poms_vec_zero_ghosts (behind V.empty()): every entry outside the interior is
    0 -- ghost planes / rows / columns and dead pitch columns -- and the interior is
    left untouched (NaN here)."""
    import ctypes as C
    import torch
    from poms_amd import _lib, runtime as rt
    from poms_amd.stencil import StencilVectorSpace
    V = StencilVectorSpace(list(npts), [p] * ndim, align=align)
    store = torch.full((V.store_elems,), float("nan"), dtype=torch.float64, device=gpu)
    _lib.call("poms_vec_zero_ghosts", V.ctx, C.byref(V.layout), rt.ptr(V.view(store)), rt.stream_handle())
    full = torch.as_strided(store, V.padded_shape[:-1] + (V.pitch,), V.strides, V.shift).cpu().numpy()
    inner = np.zeros(full.shape, dtype=bool)
    inner[tuple(slice(p, p + n) for n in npts)] = True
    assert np.all(np.isnan(full[inner]))
    assert np.all(full[~inner] == 0.0)
    v = V.empty()
    assert np.all(torch.as_strided(v._store, full.shape, V.strides, V.shift).cpu().numpy()[~inner] == 0.0)


def test_kron_dot_pyccel_2d_dropin(gpu):
    """Host-pointer drop-in vs the restated pyccel loop nest on a sub-block with ghost data."""
    from poms_amd.kron_product import kron_dot_pyccel_2d
    rng = np.random.default_rng(11)
    n1g, n2g, p1, p2 = 40, 33, 2, 3
    A = rng.uniform(-1, 1, (n1g, 2 * p1 + 1))
    B = rng.uniform(-1, 1, (n2g, 2 * p2 + 1))
    starts, ends, pads = np.array([5, 7]), np.array([30, 29]), np.array([p1, p2])
    shape = (ends[0] - starts[0] + 1 + 2 * p1, ends[1] - starts[1] + 1 + 2 * p2)
    X = rng.uniform(-1, 1, shape)
    Y = np.zeros(shape)
    Yr, Xt = np.zeros(shape), np.zeros(shape)
    kron_dot_pyccel_2d(starts, ends, pads, X, np.zeros(shape), Y, A, B)
    orc.kron_dot_pyccel_2d(starts, ends, pads, X, Xt, Yr, A, B)
    assert rel(Y, Yr) <= TOL


def test_diag_scale_and_first_sweep(gpu):
    from poms_amd.stencil import KronOperator
    p, cells = 3, (10, 12, 64)
    M, K = zip(*[_factors(p, N) for N in cells])
    npts = tuple(N + p for N in cells)
    V = _space(npts, (p,) * 3)
    A = KronOperator.laplace(V, M, K)
    b = np.random.default_rng(2).uniform(-1, 1, npts)
    out = V.empty()
    nrm = A.diag_scale(V.zeros().from_numpy(b), out, 2.0 / 3.0, want_norm=True)
    ref = (2.0 / 3.0) * b / orc.kron_sum_diag(M, K)
    assert rel(out.to_local_numpy(), ref) <= 1e-15
    assert abs(nrm - float(np.vdot(ref, ref))) <= 1e-12 * float(np.vdot(ref, ref))


@pytest.mark.parametrize("variant", [4, 7, 8, 9, 10])
@pytest.mark.parametrize("ndim,cells,p", [(3, (25, 18, 70), 3), (2, (64, 64), 3), (3, (14, 12, 66), 5)])
def test_jacobi_sweep_fused_dot(gpu, variant, ndim, cells, p):
    """poms_op_jacobi_sweep_dot: same x_out as the plain sweep, x_out.b == StencilVector.dot."""
    from poms_amd.stencil import KronOperator
    rng = np.random.default_rng(3)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    V = _space(n, [p] * ndim)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    A.set_variant(variant)
    assert A.fused_dot_supported
    x, b = V.zeros().from_numpy(rng.standard_normal(n)), V.zeros().from_numpy(rng.standard_normal(n))
    y1, y2 = V.zeros(), V.zeros()
    nrm1 = A.jacobi_sweep(b, x, y1, 2.0 / 3.0, want_norm=True)
    nrm2, dot = A.jacobi_sweep(b, x, y2, 2.0 / 3.0, want_norm=True, want_dot=True)
    np.testing.assert_array_equal(y1.to_local_numpy(), y2.to_local_numpy())
    assert abs(nrm1 - nrm2) <= 1e-14 * abs(nrm1)
    want = float(np.vdot(y1.to_local_numpy(), b.to_local_numpy()))
    assert abs(dot - want) <= 1e-12 * (abs(want) + np.linalg.norm(y1.to_local_numpy()) * np.linalg.norm(b.to_local_numpy()))
    _, dot_only = A.jacobi_sweep(b, x, y2, 2.0 / 3.0, want_norm=False, want_dot=True)
    assert abs(dot_only - dot) <= 1e-14 * abs(dot) + 1e-300
    A.set_variant(0)
    assert not A.fused_dot_supported


@pytest.mark.parametrize("variant", [8, 9, 10])
@pytest.mark.parametrize("ndim,cells,p", [(3, (25, 18, 70), 3), (3, (20, 24, 65), 2), (3, (14, 12, 66), 5),
                                          (3, (21, 33, 40), 1), (2, (64, 70), 3), (2, (150, 130), 3),
                                          (2, (40, 33), 2), (2, (37, 90), 5)])
def test_jacobi_from_zero(gpu, ndim, cells, p, variant):
    """poms_op_jacobi_from_zero == diag_scale (sweep 1) followed by one sweep, with both norms
    (2D since round 6: the v3 build, 40-row tiles at p = 3)."""
    from poms_amd.stencil import KronOperator
    rng = np.random.default_rng(5)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    V = _space(n, [p] * ndim)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    A.set_variant(variant)   # 10: v5, 8-wave tiles for the sweeps from zero
    assert A.from_zero_supported
    b = V.zeros().from_numpy(rng.standard_normal(n))
    x1, x2 = V.zeros(), V.zeros()
    n1 = A.diag_scale(b, x1, 2.0 / 3.0, want_norm=True)
    n2 = A.jacobi_sweep(b, x1, x2, 2.0 / 3.0, want_norm=True)
    y = V.zeros()
    m1, m2 = A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True)
    assert rel(y.to_local_numpy(), x2.to_local_numpy()) <= TOL
    assert abs(m1 - n1) <= 1e-12 * n1 and abs(m2 - n2) <= 1e-12 * n2
    lz = A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True, lazy=True)
    assert abs(lz.value(0) - m1) <= 1e-14 * m1 and abs(lz.value(1) - m2) <= 1e-14 * m2
    # ghosts of the output stay zero
    g = y._data.clone()
    V.interior(g).zero_()
    assert not bool(g.any())


@pytest.mark.parametrize("cells,kind,form,align", [
    ((64, 64), "spline", "sum", False),
    ((150, 130), "spline", "sum", True),     # ragged tiles on both axes
    ((7, 9), "spline", "sum", False),        # smaller than one tile
    ((1024, 1024), "spline", "sum", True),   # the 2D bench grid (22 x 20 tiles)
    ((61, 300), "random", "sum", False),     # no Toeplitz interior: band rows per row / per lane
    ((90, 70), "spline", "product", False),
    ((100, 97), "random", "product", True),
])
def test_jacobi_sweep2(gpu, cells, kind, form, align):
    """Two damped-Jacobi sweeps per launch (kron_2d.hip, epilogue 6) == two single
    v3 sweeps, bitwise over the whole storage (ghosts stay zero), into a clean and
    into a dirty output buffer; both norms (their sums group the points by the
    two-sweep kernel's tiles: equal to rounding)."""
    import torch
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    rng = np.random.default_rng(sum(cells))
    F = [_factors(p, N, rng, kind) for N in cells]
    n = [N + p for N in cells]
    V = StencilVectorSpace(n, [p, p], align=align)
    if form == "sum":
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    else:
        A = KronOperator.product(V, [f[0] for f in F])
    assert A.sweep2_supported
    b = V.zeros().from_numpy(rng.standard_normal(n))
    x0 = V.zeros().from_numpy(rng.standard_normal(n))
    x1, x2 = V.zeros(), V.zeros()
    om = 2.0 / 3.0
    n1 = A.jacobi_sweep(b, x0, x1, om, want_norm=True)
    n2 = A.jacobi_sweep(b, x1, x2, om, want_norm=True)
    y = V.zeros()
    m1, m2 = A.jacobi_sweep2(b, x0, y, om, want_norm=True)
    assert torch.equal(y._data, x2._data)
    assert abs(m1 - n1) <= 1e-12 * n1 and abs(m2 - n2) <= 1e-12 * n2
    ref = orc.kron_sum_apply if form == "sum" else None
    if ref is not None and max(cells) <= 300:   # and against the oracle's two sweeps
        xr = x0.to_local_numpy()
        M1, K1, M2, K2 = F[0][0], F[0][1], F[1][0], F[1][1]
        d1 = lambda B: B[:, p]
        D = np.outer(d1(M1) + d1(K1), d1(M2)) + np.outer(d1(M1), d1(K2))
        for _ in range(2):
            xr = xr + om * (b.to_local_numpy() - ref(xr, [f[0] for f in F], [f[1] for f in F])) / D
        assert rel(y.to_local_numpy(), xr) <= 1e-12
    y2 = V.zeros().from_numpy(rng.standard_normal(n))   # stale interior: every point is rewritten
    assert A.jacobi_sweep2(b, x0, y2, om) is None
    assert torch.equal(y2._data, x2._data)


@pytest.mark.parametrize("cells,kind", [((64, 64), "spline"), ((150, 130), "spline"), ((7, 9), "spline"),
                                        ((1024, 1024), "spline"), ((61, 300), "random")])
def test_jacobi3_from_zero(gpu, cells, kind):
    """Sweeps 1-3 from zero in one launch (epilogue 7) == the from-zero pair followed by
    one sweep, bitwise; the three norms to rounding."""
    import torch
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    rng = np.random.default_rng(sum(cells) + 1)
    F = [_factors(p, N, rng, kind) for N in cells]
    n = [N + p for N in cells]
    V = StencilVectorSpace(n, [p, p], align=True)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    b = V.zeros().from_numpy(rng.standard_normal(n))
    x2, x3 = V.zeros(), V.zeros()
    om = 2.0 / 3.0
    n1, n2 = A.jacobi_from_zero(b, x2, om, want_norm=True)
    n3 = A.jacobi_sweep(b, x2, x3, om, want_norm=True)
    y = V.zeros().from_numpy(rng.standard_normal(n))   # stale interior: every point is rewritten
    m1, m2, m3 = A.jacobi3_from_zero(b, y, om, want_norm=True)
    assert torch.equal(y._data, x3._data)
    for a, c in ((m1, n1), (m2, n2), (m3, n3)):
        assert abs(a - c) <= 1e-12 * c
    assert A.jacobi3_from_zero(b, y, om) is None
    assert torch.equal(y._data, x3._data)


def test_jacobi_sweep2_supported(gpu):
    """Two sweeps per launch: one-rank 2D p = 3 only."""
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    for nd, p in ((2, 2), (3, 3)):
        F = assemble_1d(uniform_knots(p, 20), p)
        V = StencilVectorSpace([20 + p] * nd, [p] * nd)
        A = KronOperator.laplace(V, [F[0]] * nd, [F[1]] * nd)
        assert not A.sweep2_supported
        with pytest.raises(NotImplementedError):
            A.jacobi_sweep2(V.zeros(), V.zeros(), V.zeros(), 0.5)


@pytest.mark.parametrize("variant", [4, 8, 9, 10])
@pytest.mark.parametrize("ndim,cells,p", [(3, (25, 18, 70), 3), (2, (64, 64), 3), (3, (14, 12, 66), 5)])
def test_apply_fused_inner(gpu, variant, ndim, cells, p):
    """poms_op_apply_dot: q = A p bit-identical to the apply of the same kernel family, p.q == dot."""
    from poms_amd.stencil import KronOperator
    rng = np.random.default_rng(8)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    V = _space(n, [p] * ndim)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    A.set_variant(variant)
    assert A.apply_dot_supported
    x = V.zeros().from_numpy(rng.standard_normal(n))
    q = V.zeros()
    pq = A.dot_inner(x, q)
    ref = orc.kron_sum_apply(rng.standard_normal(n) * 0 + x.to_local_numpy(), [f[0] for f in F], [f[1] for f in F])
    assert rel(q.to_local_numpy(), ref) <= TOL
    want = float(np.vdot(x.to_local_numpy(), q.to_local_numpy()))
    assert abs(pq - want) <= 1e-12 * (abs(want) + np.linalg.norm(x.to_local_numpy()) * np.linalg.norm(ref))
    A.set_variant(7)
    assert not A.apply_dot_supported


@pytest.mark.parametrize("p,cells", [(2, (20, 24, 131)), (3, (25, 18, 140)), (5, (14, 12, 100))])
@pytest.mark.parametrize("variant", [7, 8, 9, 10])
@pytest.mark.parametrize("tile_cols", [0, 48, 32])
def test_aligned_layout_and_tile_cols(gpu, p, cells, variant, tile_cols):
    """Line-aligned row pitch (poms_layout.pitch) and narrower v3/v4 tiles give the
    same apply / residual / Jacobi results as the default layout and tiles."""
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    if tile_cols > 64 - 2 * p:
        pytest.skip("tile wider than 64 - 2p")
    rng = np.random.default_rng(77 + p)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    x0, b0 = rng.standard_normal(n), rng.standard_normal(n)
    out = {}
    for align in (False, True):
        V = StencilVectorSpace(n, [p] * 3, align=align)
        assert V.aligned == align
        if align:
            assert V.pitch % 16 == 0 and (V.shift + p) % 16 == 0
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        A.set_variant(variant)
        if align:
            A.set_tile_cols(tile_cols)
        x, b = V.zeros().from_numpy(x0), V.zeros().from_numpy(b0)
        y, r, xn = V.zeros(), V.zeros(), V.zeros()
        A.dot(x, out=y)
        A.residual(b, x, out=r)
        nrm = A.jacobi_sweep(b, x, xn, 2.0 / 3.0, want_norm=True)
        out[align] = (y.toarray(), r.toarray(), xn.toarray(), nrm)
    for k in range(3):
        assert rel(out[True][k], out[False][k]) <= 1e-14, k
    assert abs(out[True][3] - out[False][3]) <= 1e-12 * abs(out[False][3])


@pytest.mark.gpu
def test_native_comm_single_rank(gpu):
    """poms_comm_* on a one-rank RCCL communicator: the all-reduce is the identity,
    a ghost exchange without neighbours is a no-op, the streams stay ordered."""
    import ctypes as C
    import torch
    from poms_amd import _lib
    from poms_amd.dist import NativeComm
    from poms_amd import runtime as rt
    nb = _lib.lib.poms_comm_id_bytes()
    buf = C.create_string_buffer(nb)
    _lib.call("poms_comm_unique_id", buf, nb)
    h = C.c_void_p()
    _lib.call("poms_comm_create", 0, C.c_char_p(bytes(buf.raw[:nb])), 0, 1, C.byref(h))
    try:
        nc = NativeComm(h, 0)
        t = torch.arange(5, dtype=torch.float64, device=gpu) + 0.5
        nc.allreduce(t, rt.stream_handle(), wait_back=True)
        assert torch.equal(t.cpu(), torch.arange(5, dtype=torch.float64) + 0.5)
        assert nc._self_test(0, 1)
        # result ready on the communication stream only (wait_back = False)
        u = torch.full((3,), 2.0, dtype=torch.float64, device=gpu)
        nc.allreduce(u, rt.stream_handle(), wait_back=False)
        nc.stream.synchronize()
        assert torch.equal(u.cpu(), torch.full((3,), 2.0, dtype=torch.float64))
    finally:
        _lib.call("poms_comm_destroy", h)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [9, 10])
def test_two_range_launch(gpu, variant):
    """poms_op_run_reduce2: interior planes, then both p-plane boundaries in ONE launch
    (the overlapped slab schedule) == one launch over all planes, norms included."""
    import torch
    from poms_amd import _lib, runtime as rt
    from poms_amd.stencil import KronOperator
    p, cells = 3, (20, 18, 70)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    V = _space(n, [p] * 3)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    A.set_variant(variant)
    rng = np.random.default_rng(21)
    x, b = V.zeros().from_numpy(rng.standard_normal(n)), V.zeros().from_numpy(rng.standard_normal(n))
    y1, y2 = V.zeros(), V.zeros()
    nb = torch.zeros(8, dtype=torch.float64, device=gpu)
    st = rt.stream_handle()
    n0 = n[0]
    for kind, epi in (("apply", 0), ("jacobi", 2)):
        wn = epi == 2
        _lib.call("poms_op_run_reduce2", A._h, epi, 2.0 / 3.0, rt.ptr(x._data), rt.ptr(y1._data), rt.ptr(b._data),
                  0, n0, 0, 0, rt.ptr(nb[0:1]) if wn else None, None, 0, st)
        _lib.call("poms_op_run_reduce2", A._h, epi, 2.0 / 3.0, rt.ptr(x._data), rt.ptr(y2._data), rt.ptr(b._data),
                  p, n0 - p, 0, 0, rt.ptr(nb[1:2]) if wn else None, None, 0, st)
        _lib.call("poms_op_run_reduce2", A._h, epi, 2.0 / 3.0, rt.ptr(x._data), rt.ptr(y2._data), rt.ptr(b._data),
                  0, p, n0 - p, n0, rt.ptr(nb[1:2]) if wn else None, None, 1, st)
        np.testing.assert_array_equal(y1.to_local_numpy(), y2.to_local_numpy())
        if wn:
            h = nb.cpu()
            assert abs(float(h[0]) - float(h[1])) <= 1e-13 * abs(float(h[0])), kind


@pytest.mark.gpu
def test_native_comm_lazy_slot(gpu):
    """The native ring slot path of a lazily read norm (one rank): the sweep reduces
    into the host-mapped slot, poms_allreduce_to_host registers it, value() waits for
    it (and leaves the sum in the pinned destination)."""
    import ctypes as C
    from poms_amd import _lib, runtime as rt
    from poms_amd.dist import NativeComm
    from poms_amd.stencil import KronOperator
    nbytes = _lib.lib.poms_comm_id_bytes()
    buf = C.create_string_buffer(nbytes)
    _lib.call("poms_comm_unique_id", buf, nbytes)
    h = C.c_void_p()
    _lib.call("poms_comm_create", 0, C.c_char_p(bytes(buf.raw[:nbytes])), 0, 1, C.byref(h))
    try:
        nc = NativeComm(h, 0)
        p, cells = 3, (12, 14, 40)
        F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
        n = [N + p for N in cells]
        V = _space(n, [p] * 3)
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        rng = np.random.default_rng(5)
        x, b = V.zeros().from_numpy(rng.standard_normal(n)), V.zeros().from_numpy(rng.standard_normal(n))
        ref = A.jacobi_sweep(b, x, V.zeros(), 2.0 / 3.0, want_norm=True)
        for _ in range(20):   # wraps the 16-slot ring
            slot, ticket = nc.slot()
            A._run("jacobi", x, V.zeros(), b=b, omega=2.0 / 3.0, norm_out=slot)
            lz = nc.to_host(ticket, 1, V.pinned_slots(1), rt.stream_handle())
            assert abs(lz.value() - ref) <= 1e-13 * ref
    finally:
        _lib.call("poms_comm_destroy", h)


@pytest.mark.gpu
def test_native_run_dist_single_rank(gpu):
    """poms_op_run_dist on a one-rank communicator (no neighbours): the overlapped
    schedule (interior, then both boundaries) and its device / lazy reductions equal
    one plain launch."""
    import ctypes as C
    import torch
    from poms_amd import _lib, runtime as rt
    from poms_amd.dist import LazyNative, NativeComm
    from poms_amd.stencil import KronOperator
    nbytes = _lib.lib.poms_comm_id_bytes()
    buf = C.create_string_buffer(nbytes)
    _lib.call("poms_comm_unique_id", buf, nbytes)
    h = C.c_void_p()
    _lib.call("poms_comm_create", 0, C.c_char_p(bytes(buf.raw[:nbytes])), 0, 1, C.byref(h))
    try:
        nc = NativeComm(h, 0)
        p, cells = 3, (21, 14, 40)
        F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
        n = [N + p for N in cells]
        V = _space(n, [p] * 3)
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        rng = np.random.default_rng(6)
        x, b = V.zeros().from_numpy(rng.standard_normal(n)), V.zeros().from_numpy(rng.standard_normal(n))
        y_ref = V.zeros()
        ref = A.jacobi_sweep(b, x, y_ref, 2.0 / 3.0, want_norm=True)
        dev = torch.zeros(2, dtype=torch.float64, device=gpu)
        for lazy in (0, 1):
            y = V.zeros()
            host = V.pinned_slots(1)
            tk = C.c_int(-1)
            _lib.call("poms_op_run_dist", A._h, nc.h, 2, 2.0 / 3.0, rt.ptr(x._data), rt.ptr(y._data), rt.ptr(b._data),
                      C.c_void_p(V.planes(x._store).data_ptr()), V.plane_elems, V.local_npts[0], V.pads[0], p,
                      -1, -1, 1, 1, 0, None if lazy else rt.ptr(dev[0:1]), None, lazy,
                      C.c_void_p(host.data_ptr()) if lazy else None, C.byref(tk), rt.stream_handle())
            np.testing.assert_array_equal(y.to_local_numpy(), y_ref.to_local_numpy())
            got = LazyNative(nc, tk.value, host).value() if lazy else float(dev[0].item())
            assert abs(got - ref) <= 1e-13 * ref, lazy
    finally:
        _lib.call("poms_comm_destroy", h)


@pytest.mark.parametrize("p,cells,align", [(1, (21, 33, 150), False), (2, (20, 24, 131), True),
                                           (2, (20, 24, 131), False), (3, (25, 140, 140), True),
                                           (3, (25, 18, 140), True), (3, (25, 18, 140), False),
                                           (3, (40, 70, 250), True)])
def test_v5_jacobi_from_zero_coverage(gpu, p, cells, align):
    """Two sweeps from zero on v5 (16-wave tiles at p <= 3; wide axis 2 -> several
    128-column tiles, aligned and unaligned layouts, a two-range launch) against
    diag_scale + one sweep, and the default selection picks v5 for it."""
    import torch
    from poms_amd import _lib, runtime as rt
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    rng = np.random.default_rng(40 + p)
    F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
    n = [N + p for N in cells]
    V = StencilVectorSpace(n, [p] * 3, align=align)
    A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
    A.set_variant(8)
    # the default picks v5 for every case: at p = 3 16-wave tiles when axes 1 and 2
    # share their Toeplitz rows (equal cell counts), 8-wave tiles otherwise (round 6;
    # v3 took those before)
    want = 10
    assert A.kernel_variant("jacobi_from_zero") == want
    A.set_variant(10)
    assert A.kernel_variant("jacobi_from_zero") == want
    b = V.zeros().from_numpy(rng.standard_normal(n))
    x1, x2 = V.zeros(), V.zeros()
    n1 = A.diag_scale(b, x1, 2.0 / 3.0, want_norm=True)
    n2 = A.jacobi_sweep(b, x1, x2, 2.0 / 3.0, want_norm=True)
    y = V.zeros()
    m1, m2 = A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True)
    assert rel(y.to_local_numpy(), x2.to_local_numpy()) <= TOL
    assert abs(m1 - n1) <= 1e-12 * n1 and abs(m2 - n2) <= 1e-12 * n2
    # interior planes, then both p-plane boundaries in one launch == one launch
    y2 = V.zeros()
    nb = torch.zeros(4, dtype=torch.float64, device=gpu)
    st = rt.stream_handle()
    n0 = n[0]
    _lib.call("poms_op_run_reduce2", A._h, 3, 2.0 / 3.0, rt.ptr(b._data), rt.ptr(y2._data), rt.ptr(b._data),
              p, n0 - p, 0, 0, rt.ptr(nb[1:2]), rt.ptr(nb[0:1]), 0, st)
    _lib.call("poms_op_run_reduce2", A._h, 3, 2.0 / 3.0, rt.ptr(b._data), rt.ptr(y2._data), rt.ptr(b._data),
              0, p, n0 - p, n0, rt.ptr(nb[1:2]), rt.ptr(nb[0:1]), 1, st)
    np.testing.assert_array_equal(y2.to_local_numpy(), y.to_local_numpy())
    h = nb.cpu()
    assert abs(float(h[0]) - m1) <= 1e-13 * m1 and abs(float(h[1]) - m2) <= 1e-13 * m2


@pytest.mark.parametrize("p", [1, 2, 3])
@pytest.mark.parametrize("variant", [0, 4, 7, 8, 9, 10])
def test_block_with_ghost_data(gpu, p, variant):
    """A block of a decomposition of axes 1 and 2 (spl Cart): the owned rows are a
    window [s, s + n) of larger global factors and the ghost rows / columns --
    edges and corners included -- hold the neighbours' values.  Every variant must
    read them (the operator is told with poms_op_set_ghost_corners; v5 at odd p,
    which drops the corner ghost, is not selected then)."""
    from poms_amd import _lib
    from poms_amd.stencil import StencilVectorSpace, KronOperator, _widen
    import ctypes as C
    rng = np.random.default_rng(90 + p)
    cells_g = (14, 40, 150)
    Mg, Kg = zip(*[assemble_1d(uniform_knots(p, N), p) for N in cells_g])
    ng = [N + p for N in cells_g]
    s1, s2 = 11, 23                       # block offsets on axes 1 and 2
    nl = (ng[0], 17, 100)                 # axis 0 whole, axes 1 and 2 a window
    xg = rng.standard_normal(ng)
    V = StencilVectorSpace(list(nl), [p] * 3)
    # operator whose axis-1/2 factor rows are the window's rows (as a Cart block)
    bands = {"A0": Mg[0] + Kg[0], "M0": Mg[0], "A1": Mg[1][s1:s1 + nl[1]], "B1": Kg[1][s1:s1 + nl[1]],
             "M2": Mg[2][s2:s2 + nl[2]], "K2": Kg[2][s2:s2 + nl[2]]}
    A = KronOperator(V, "sum", {k: _widen(v, p) for k, v in bands.items()}, p)
    _lib.call("poms_op_set_ghost_corners", A._h, 1)
    A.set_variant(variant)
    if p & 1:
        assert A.kernel_variant("apply") != 10
    x = V.zeros()
    win = np.zeros(V.padded_shape)
    win[p:p + nl[0]] = xg[:, s1 - p:s1 + nl[1] + p, s2 - p:s2 + nl[2] + p]
    x._data.copy_(torch_from(win))
    y = A.dot(x).to_local_numpy()
    ref = orc.kron_sum_apply(xg, Mg, Kg)[:, s1:s1 + nl[1], s2:s2 + nl[2]]
    assert rel(y, ref) <= TOL
    # the same operator without the declaration keeps v5 at odd p (corner ghost zero)
    if p & 1 and variant in (8, 10):
        _lib.call("poms_op_set_ghost_corners", A._h, 0)
        assert A.kernel_variant("apply") == 10


def torch_from(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a))

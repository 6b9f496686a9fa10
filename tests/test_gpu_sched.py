"""The v5 dispatch order (``poms_diag_v5_sched``, ``KronGeom::sched`` in csrc/kron_v5.hip):
each XCD starts its range of tiles longest-estimated first.  The order only moves
work between CUs: every output and every norm (the partial sums keep their slots
in the default order) must equal the default order's bitwise, for the operator
calls of the damped-Jacobi smoother (`sources/solvers.py:197-222`) and the
mat-vec (`pyccel/pyccel_functions.py:4-21`)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sched(mode):
    from poms_amd import _lib
    return _lib.lib.poms_diag_v5_sched(mode)


@pytest.mark.parametrize("cells,align", [(20, True), (45, False), (109, True), (140, False)])
def test_dispatch_order_is_bitwise_neutral(cells, align):
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    p = 3
    M, K = assemble_1d(uniform_knots(p, cells), p)
    n = cells + p
    V = StencilVectorSpace([n] * 3, [p] * 3, align=align)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    A.set_variant(10)
    gen = torch.Generator(device="cuda").manual_seed(cells)
    x, b = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1, generator=gen)
    V.interior(b._data).uniform_(-1, 1, generator=gen)
    prev = _sched(-1)
    res = []
    try:
        for mode in (0, 1):
            assert _sched(mode) in (0, 1)
            y, r, xo, j0 = V.zeros(), V.zeros(), V.zeros(), V.zeros()
            A.dot(x, out=y)
            A.residual(b, x, out=r)
            n1 = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
            n0 = A.jacobi_from_zero(b, j0, 2.0 / 3.0, want_norm=True)
            ad = float(A.dot_inner(x, V.zeros(), device=True))
            torch.cuda.synchronize()
            assert A.last_variant == 10
            res.append(([t._data.clone() for t in (y, r, xo, j0)], (n1, n0, ad)))
    finally:
        _sched(prev)
    for u, v in zip(res[0][0], res[1][0]):
        assert torch.equal(u, v)
    assert res[0][1] == res[1][1], res


def test_dispatch_order_toggle_returns_previous_mode():
    prev = _sched(-1)
    try:
        assert _sched(0) == prev
        assert _sched(1) == 0
        assert _sched(-1) == 1
    finally:
        _sched(prev)

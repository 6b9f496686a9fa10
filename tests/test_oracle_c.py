"""The C restatement (oracle/kron_cpu.c, the CPU baseline) against the NumPy oracle."""
import numpy as np
import pytest

from oracle import cpu_baseline as cb
from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, uniform_knots


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


@pytest.mark.parametrize("p,N", [(1, 6), (2, 9), (3, 12), (5, 11)])
def test_c_kron_sum_modes(p, N):
    M, K = assemble_1d(uniform_knots(p, N), p)
    A = cb.CpuLaplace3D(M, K, p)
    n = A.n
    rng = np.random.default_rng(p)
    x, b = A.zeros(), A.zeros()
    sl = (slice(p, p + n),) * 3
    x[sl] = rng.standard_normal((n,) * 3)
    b[sl] = rng.standard_normal((n,) * 3)
    y_ref = orc.kron_sum_apply(x[sl], [M] * 3, [K] * 3)
    assert rel(A.dot(x)[sl], y_ref) <= 1e-14
    assert rel(A.residual(b, x)[sl], b[sl] - y_ref) <= 1e-14
    D = orc.kron_sum_diag([M] * 3, [K] * 3)
    xo, nrm = A.jacobi_sweep(b, x, 2.0 / 3.0)
    dr = 2.0 / 3.0 * (b[sl] - y_ref) / D
    assert rel(xo[sl], x[sl] + dr) <= 1e-14
    assert abs(nrm - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr))
    # ghost cells of the outputs stay zero
    y = A.dot(x)
    y[sl] = 0
    assert not y.any()
    assert abs(A.vdot(x, b) - float(np.vdot(x[sl], b[sl]))) <= 1e-12 * n ** 1.5
    np.testing.assert_allclose(A.axpby(2.0, x, -0.5, b)[sl], 2 * x[sl] - 0.5 * b[sl], rtol=0, atol=1e-15)


def test_c_vcycle_matches_numpy_oracle():
    """cpu_baseline's V-cycle schedule (incl. the discarded A.dot) == poms_oracle.vcycle_two_level (p=2)."""
    from poms_amd.splines import matrix_multi_stages
    p, N, Nc = 2, 12, 4
    r = cb.time_vcycle(N=N, p=p, Nc=Nc, cycles=1, threads=2)
    assert r["dof"] == (N + p) ** 3
    Tc, Tf = uniform_knots(p, Nc), uniform_knots(p, N)
    nf, nc = N + p, Nc + p
    P1 = matrix_multi_stages(orc.knots_to_insert(Tf, nf, p, Tc, nc, p), nc, p, Tc)
    M, K = assemble_1d(Tf, p)
    _, ipre, ipos = orc.vcycle_two_level([M] * 3, [K] * 3, P1, np.ones((nf,) * 3))
    _, _, ipos2 = orc.vcycle_two_level([M] * 3, [K] * 3, P1, np.ones((nf,) * 3), reorder=True)
    assert r["info_pre"]["niter"] == ipre["niter"] and r["info_pos"]["niter"] == ipos["niter"]
    # the final residual sits at roundoff level (|x| ~ 1e5, ||r|| ~ 1e-3, i.e. 1e-8 of the
    # scale): two summation orders of the same oracle already differ by percents, so only
    # its order of magnitude is compared
    assert ipos2["niter"] == ipos["niter"]
    assert 0.5 * ipos["res_norm"] <= r["info_pos"]["res_norm"] <= 2.0 * ipos["res_norm"]

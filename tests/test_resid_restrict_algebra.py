"""CPU check of the factorisation poms_resid_restrict evaluates:

    R (b - A x) = R b - (R A) x,   A = A0⊗A1⊗M2 + M0⊗B1⊗M2 + M0⊗A1⊗K2  (FORM_SUM, 3D)
    u_c = P0ᵀ b, u_a = G_A0ᵀ x, u_m = G_M0ᵀ x                      (axis 0)
    v_3 = P1ᵀ u_c, v_1 = G_A1ᵀ u_a + G_B1ᵀ u_m, v_2 = G_A1ᵀ u_m     (axis 1)
    rc  = P2ᵀ v_3 - G_M2ᵀ v_1 - G_K2ᵀ v_2                          (axis 2)

with G = Fᵀ P per 1D factor, against the materialised R (b - A x) of the reference's
`sources/mg_jac.py:93-94` (scipy.sparse Kronecker products).  The same pass structure
for 2D (A1⊗M2 + B1⊗K2) and FORM_SINGLE.  No GPU: the pass/role wiring of the C code
restated in numpy.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from poms_amd.mg import two_level_setup_1d
from poms_amd.splines import assemble_1d, band_to_dense, uniform_knots


def _axis(T, G, axis):
    """Contract ``axis`` of T with G (rows: fine index, columns: coarse)."""
    return np.moveaxis(np.tensordot(T, G, axes=([axis], [0])), -1, axis)


@pytest.mark.parametrize("p,Nf,Nc,c", [(3, 32, 8, 1.0), (2, 24, 4, 0.5), (1, 16, 8, 2.0)])
def test_sum_form_3d(p, Nf, Nc, c):
    M, K = assemble_1d(uniform_knots(p, Nf), p)
    _, _, P = two_level_setup_1d(p, uniform_knots(p, Nf), uniform_knots(p, Nc))
    Md, Kd = band_to_dense(M), band_to_dense(K)
    roles = {"A0": c * Md + Kd, "M0": Md, "A1": Md, "B1": Kd, "M2": Md, "K2": Kd}
    G = {k: v.T @ P for k, v in roles.items()}
    n = Md.shape[0]
    rng = np.random.default_rng(1)
    x, b = rng.standard_normal((n,) * 3), rng.standard_normal((n,) * 3)
    # the passes
    u_c, u_a, u_m = _axis(b, P, 0), _axis(x, G["A0"], 0), _axis(x, G["M0"], 0)
    v3 = _axis(u_c, P, 1)
    v1 = _axis(u_a, G["A1"], 1) + _axis(u_m, G["B1"], 1)
    v2 = _axis(u_m, G["A1"], 1)
    rc = _axis(v3, P, 2) - _axis(v1, G["M2"], 2) - _axis(v2, G["K2"], 2)
    # the reference: materialised operator, residual, restriction
    S = lambda m: sp.csr_matrix(m)
    A = (sp.kron(sp.kron(S(roles["A0"]), S(Md)), S(Md)) + sp.kron(sp.kron(S(Md), S(Kd)), S(Md))
         + sp.kron(sp.kron(S(Md), S(Md)), S(Kd)))
    R = sp.kron(sp.kron(S(P.T), S(P.T)), S(P.T))
    want = R @ (b.reshape(-1) - A @ x.reshape(-1))
    assert np.linalg.norm(rc.reshape(-1) - want) <= 1e-12 * np.linalg.norm(want)


@pytest.mark.parametrize("form", ["sum", "single"])
def test_2d_and_single(form):
    p, Nf, Nc = 3, 48, 8
    M, K = assemble_1d(uniform_knots(p, Nf), p)
    _, _, P = two_level_setup_1d(p, uniform_knots(p, Nf), uniform_knots(p, Nc))
    Md, Kd = band_to_dense(M), band_to_dense(K)
    n = Md.shape[0]
    rng = np.random.default_rng(2)
    x, b = rng.standard_normal((n, n)), rng.standard_normal((n, n))
    if form == "sum":   # A = A1⊗M2 + B1⊗K2
        F1a, F1b, F2a, F2b = 0.75 * Md + Kd, Md, Md, Kd
        u_c, u_a, u_m = _axis(b, P, 0), _axis(x, F1a.T @ P, 0), _axis(x, F1b.T @ P, 0)
        rc = _axis(u_c, P, 1) - _axis(u_a, F2a.T @ P, 1) - _axis(u_m, F2b.T @ P, 1)
        A = sp.kron(sp.csr_matrix(F1a), sp.csr_matrix(F2a)) + sp.kron(sp.csr_matrix(F1b), sp.csr_matrix(F2b))
    else:               # A = F1⊗F2
        F1, F2 = Md + 0.1 * Kd, Kd + 0.2 * Md
        u_c, u_a = _axis(b, P, 0), _axis(x, F1.T @ P, 0)
        rc = _axis(u_c, P, 1) - _axis(u_a, F2.T @ P, 1)
        A = sp.kron(sp.csr_matrix(F1), sp.csr_matrix(F2))
    R = sp.kron(sp.csr_matrix(P.T), sp.csr_matrix(P.T))
    want = R @ (b.reshape(-1) - A @ x.reshape(-1))
    assert np.linalg.norm(rc.reshape(-1) - want) <= 1e-12 * np.linalg.norm(want)

"""Pin the CPU oracle (and the host-side set-up) to the reference's own outputs.

Fixtures in tests/golden/*.npz were produced by tests/golden/make_golden.py,
which imports the reference's Python (pyccel_functions, utils, solvers,
matrix_assembler, multilevels) and runs its mg_jac.py driver, with the build's
spl stand-in for the absent third-party spl package.
"""
import numpy as np
import pytest

from oracle import poms_oracle as orc
from poms_amd.splines import assemble_1d, make_open_knots, matrix_multi_stages


def load(golden_dir, name):
    z = np.load(golden_dir / name, allow_pickle=False)
    out = {}
    for k in z.files:
        case, field = k.split("__", 1)
        out.setdefault(case, {})[field] = z[k]
    return out


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


# --------------------------------------------------------------------------- kron dot
def test_kron_dot_pyccel_2d_matches_reference(golden_dir):
    """Oracle restatement of `pyccel/pyccel_functions.py:4-21` == reference output, bit for bit."""
    cases = load(golden_dir, "kron_dot_2d.npz")
    assert len(cases) >= 13
    for name, c in cases.items():
        Y = np.zeros_like(c["Y"])
        Xt = np.zeros_like(c["X"])
        orc.kron_dot_pyccel_2d(c["starts"], c["ends"], c["pads"], c["X"], Xt, Y, c["A"], c["B"])
        np.testing.assert_array_equal(Y, c["Y"], err_msg=name)


def test_kron_dot_recipe_vs_scipy_kron(golden_dir):
    """`test_kron_dot.py` recipe (8x4, p=(2,1)): pyccel kernel == scipy.sparse.kron reference (utils.kron_dot_ref)."""
    c = load(golden_dir, "kron_dot_2d.npz")["recipe"]
    p1, p2 = c["pads"]
    n1, n2 = c["ends"] + 1
    inner = c["Y"][p1:p1 + n1, p2:p2 + n2].reshape(-1)
    assert rel(inner, c["Y_kron_ref"]) <= 1e-15
    # and the oracle's own Kronecker product apply on the unpadded grid
    X = c["X"][p1:p1 + n1, p2:p2 + n2]
    assert rel(orc.kron_product_apply(X, [c["A"], c["B"]]).reshape(-1), c["Y_kron_ref"]) <= 1e-15


def test_kron_dot_c_oracle_matches_reference(golden_dir):
    from oracle import cpu_baseline as cb
    import ctypes as C
    lib = cb.lib()
    for name, c in load(golden_dir, "kron_dot_2d.npz").items():
        st = np.ascontiguousarray(c["starts"], dtype=np.int64)
        en = np.ascontiguousarray(c["ends"], dtype=np.int64)
        pd = np.ascontiguousarray(c["pads"], dtype=np.int64)
        X = np.ascontiguousarray(c["X"])
        A, B = np.ascontiguousarray(c["A"]), np.ascontiguousarray(c["B"])
        Y, Xt = np.zeros_like(X), np.zeros_like(X)
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        lib.oracle_kron_dot_pyccel_2d(p(st), p(en), p(pd), p(X), p(Xt), p(Y), p(A), p(B))
        assert rel(Y, c["Y"]) <= 1e-15, name


# --------------------------------------------------------------------------- assembly
def test_assembly_2d_is_kronecker_sum(golden_dir):
    """Reference `assembly_2d` stencil == M⊗M + K⊗M + M⊗K from our 1D factors (SURVEY §0 probe: 3e-16)."""
    for name, c in load(golden_dir, "assembly_2d.npz").items():
        p = int(c["p"])
        ne = [int(v) for v in c["ne"]]
        F = [assemble_1d(make_open_knots(p, n + p), p) for n in ne]
        (M1, K1), (M2, K2) = F
        sten = c["stencil"]
        n1, n2 = ne[0] + p, ne[1] + p
        ref = np.zeros((n1, n2, 2 * p + 1, 2 * p + 1))
        ref += np.einsum("ik,jl->ijkl", M1, M2) + np.einsum("ik,jl->ijkl", K1, M2) + np.einsum("ik,jl->ijkl", M1, K2)
        got = sten[p:p + n1, p:p + n2]
        scale = np.max(np.abs(ref))
        assert np.max(np.abs(got - ref)) <= 1e-13 * scale, name
        np.testing.assert_array_equal(c["stencil_seq"], sten)   # assembly_2d_seq == assembly_2d on one rank
        m1 = c["mass1d"]
        assert np.max(np.abs(m1 - M1)) <= 1e-14 * np.max(np.abs(M1)), name


# --------------------------------------------------------------------------- multilevel
def test_knots_to_insert(golden_dir):
    from poms_amd.multilevels import knots_to_insert as prod_kti
    for name, c in load(golden_dir, "knots_to_insert.npz").items():
        p, nc, nf = (int(v) for v in name.replace("p", "").replace("nc", " ").replace("nf", " ").replace("_", "").split())
        got_o = orc.knots_to_insert(c["Tf"], nf, p, c["Tc"], nc, p)
        got_p = prod_kti(c["Tf"], nf, p, c["Tc"], nc, p)
        np.testing.assert_array_equal(got_o, c["ts"], err_msg=name)
        np.testing.assert_array_equal(got_p, c["ts"], err_msg=name)


def test_multi_stage_matrix_matches_driver_golden(golden_dir):
    """P1 from our restatement == the matrix the mg_jac.py golden run used (built by the same restatement in
    the spl stand-in); both pinned by the property tests in test_splines.py."""
    for name, c in load(golden_dir, "vcycle_mg_jac.npz").items():
        p = int(c["p"])
        nc = len(c["Tc"]) - p - 1
        P1 = matrix_multi_stages(c["Ts"], nc, p, c["Tc"])
        assert np.max(np.abs(P1 - c["P1"])) <= 1e-15, name


# --------------------------------------------------------------------------- solvers
def _golden_operator(golden_dir, p, ne):
    asm = load(golden_dir, "assembly_2d.npz")[f"p{p}_{ne}x{ne}"]
    sten = asm["stencil"]
    n = ne + p
    rows, cols, vals = [], [], []
    for i1 in range(n):
        for i2 in range(n):
            for k1 in range(2 * p + 1):
                for k2 in range(2 * p + 1):
                    j1, j2 = i1 + k1 - p, i2 + k2 - p
                    if 0 <= j1 < n and 0 <= j2 < n and sten[i1 + p, i2 + p, k1, k2] != 0.0:
                        rows.append(i1 * n + i2)
                        cols.append(j1 * n + j2)
                        vals.append(sten[i1 + p, i2 + p, k1, k2])
    import scipy.sparse as sp
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n * n, n * n))
    D = sten[p:p + n, p:p + n, p, p].reshape(-1)
    return A, D


@pytest.mark.parametrize("p,ne", [(1, 4), (1, 16), (3, 8)])
def test_oracle_solvers_match_reference(golden_dir, p, ne):
    """Oracle pcg / damped_jacobi / jacobi (`sources/solvers.py`) == reference on the reference's own matrix."""
    A, D = _golden_operator(golden_dir, p, ne)
    apply = lambda v: A @ v
    sol = load(golden_dir, "solvers_2d.npz")
    for rhs in ("manuf", "ones"):
        c = sol[f"p{p}_ne{ne}_{rhs}"]
        b = c["b"]
        for m in (1, 3, 10):
            x = orc.damped_jacobi(apply, D, b, tol=0.0, maxiter=m)
            assert rel(x, c[f"djac_m{m}_tol0"]) <= 1e-12
        assert rel(orc.damped_jacobi(apply, D, b), c["djac_default"]) <= 1e-12
        assert rel(orc.jacobi(D, b), c["jacobi"]) <= 1e-15
        psolve = lambda r: orc.damped_jacobi(apply, D, r)
        for m in (1, 2, 5):
            x, info = orc.pcg(apply, psolve, b, tol=0.0, maxiter=m)
            ref_info = c[f"pcg_m{m}_tol0_info"]
            assert info["niter"] == int(ref_info[0])
            assert rel(x, c[f"pcg_m{m}_tol0"]) <= 1e-10
        x, info = orc.pcg(apply, psolve, b, tol=1e-6, maxiter=10)
        ref_info = c["pcg_mgjac_info"]
        assert info["niter"] == int(ref_info[0]) and info["success"] == bool(ref_info[1])
        assert rel(x, c["pcg_mgjac"]) <= 1e-9
        for m in (3, 1000):                      # conjugate residual (`sources/solvers.py:3-65`)
            x, info = orc.crl(apply, b, tol=0.0 if m == 3 else 1e-5, maxiter=m)
            ref_info = c[f"crl_m{m}_info"]
            assert info["niter"] == int(ref_info[0]) and info["success"] == bool(ref_info[1]), (rhs, m)
            assert rel(x, c[f"crl_m{m}"]) <= (1e-10 if m == 3 else 1e-8), (rhs, m)


def test_oracle_vcycle_matches_mg_jac(golden_dir):
    """Oracle two-level V-cycle == the reference driver `sources/mg_jac.py` (run as a script)."""
    for name, c in load(golden_dir, "vcycle_mg_jac.npz").items():
        p = int(c["p"])
        T = c["T"]
        M, K = assemble_1d(T, p)
        n = len(T) - p - 1
        xr, ipre, ipos = orc.vcycle_two_level([M, M], [K, K], c["P1"], np.ones((n, n)))
        assert ipre["niter"] == int(c["info_pre"][0]) and ipos["niter"] == int(c["info_pos"][0]), name
        assert rel(xr.reshape(-1), c["xf2"]) <= 1e-8, name

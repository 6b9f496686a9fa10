"""General stencil operator (spl `StencilMatrix.dot` with per-row coefficients):
the reference's own assembled `assembly_2d` stencils (tests/golden/assembly_2d.npz)
applied on the GPU, the reference solvers run on them (solvers_2d.npz), and
random 2D/3D stencils through every epilogue against NumPy."""
import numpy as np
import pytest

from oracle import poms_oracle as orc

pytestmark = pytest.mark.gpu


def load(golden_dir, name):
    z = np.load(golden_dir / name, allow_pickle=False)
    out = {}
    for k in z.files:
        case, field = k.split("__", 1)
        out.setdefault(case, {})[field] = z[k]
    return out


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def _check_crl(info, ref, x, xref, m, rhs):
    """Fixed-count CR iterates agree to 1e-10.  Run to convergence (tol = 1e-5 on
    s.r, `sources/solvers.py:38`) the stop test reads a quantity near its
    threshold, so 1-ulp operator differences can move the stop by one iteration;
    the converged iterates then agree to the solver tolerance."""
    assert info["success"] == bool(ref[1]), (rhs, m)
    if m == 3:
        assert info["niter"] == int(ref[0]), (rhs, m)
        assert rel(x, xref) <= 1e-10, (rhs, m)
    else:
        assert abs(info["niter"] - int(ref[0])) <= 1, (rhs, m, info["niter"], ref[0])
        assert rel(x, xref) <= 1e-6, (rhs, m)


def stencil_dot_ref(data, x, pads):
    """v[i] = sum_k M[i, k] x[i + k - p] on global arrays (`slides/content.tex:285-290`)."""
    nd = x.ndim
    n = x.shape
    xp = np.pad(x, [(p, p) for p in pads])
    inner = data[tuple(slice(p, p + m) for p, m in zip(pads, n))]
    out = np.zeros(n)
    for kk in np.ndindex(*[2 * p + 1 for p in pads]):
        out += inner[(Ellipsis,) + kk] * xp[tuple(slice(k, k + m) for k, m in zip(kk, n))]
    return out


def test_assembly_2d_stencil_dot_golden(gpu, golden_dir):
    """The reference's assembled operator (`sources/matrix_assembler.py:84-179`) applied by the
    general-stencil kernel == the same stencil applied on the host."""
    from poms_amd.stencil import StencilMatrix, StencilVectorSpace
    for name, c in load(golden_dir, "assembly_2d.npz").items():
        p = int(c["p"])
        data = c["stencil"]
        n = tuple(s - 2 * p for s in data.shape[:2])
        V = StencilVectorSpace(list(n), [p, p])
        A = StencilMatrix.from_data(V, data)
        x = np.random.default_rng(p).uniform(-1, 1, n)
        y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
        assert rel(y, stencil_dot_ref(data, x, (p, p))) <= 1e-14, name
        assert rel(y.reshape(-1), A.tosparse() @ x.reshape(-1)) <= 1e-14, name


@pytest.mark.parametrize("p,ne", [(1, 4), (1, 16), (3, 8)])
def test_solvers_on_assembled_stencil_golden(gpu, golden_dir, p, ne):
    """pcg / damped_jacobi / jacobi / crl with A = the reference's assembled StencilMatrix
    == `sources/solvers.py` run by the reference on that same matrix."""
    from poms_amd.solvers import crl, damped_jacobi, jacobi, pcg
    from poms_amd.stencil import StencilMatrix, StencilVectorSpace
    st = load(golden_dir, "assembly_2d.npz")[f"p{p}_{ne}x{ne}"]["stencil"]
    n = ne + p
    V = StencilVectorSpace([n, n], [p, p])
    A = StencilMatrix.from_data(V, st)
    assert A.fused_dot_supported and A.apply_dot_supported and not A.from_zero_supported
    sol = load(golden_dir, "solvers_2d.npz")
    for rhs in ("manuf", "ones"):
        c = sol[f"p{p}_ne{ne}_{rhs}"]
        b = V.zeros().from_numpy(c["b"].reshape(n, n))
        for m in (1, 3, 10):
            x = damped_jacobi(A, b, tol=0.0, maxiter=m)
            assert rel(x.toarray(), c[f"djac_m{m}_tol0"]) <= 1e-12, (rhs, m)
        assert rel(damped_jacobi(A, b).toarray(), c["djac_default"]) <= 1e-12
        assert rel(jacobi(A, b).toarray(), c["jacobi"]) <= 1e-14
        for m in (1, 2, 5):
            x, info = pcg(A, damped_jacobi, b, tol=0.0, maxiter=m)
            assert info["niter"] == int(c[f"pcg_m{m}_tol0_info"][0])
            assert rel(x.toarray(), c[f"pcg_m{m}_tol0"]) <= 1e-10, (rhs, m)
        x, info = pcg(A, damped_jacobi, b, tol=1e-6, maxiter=10)
        ref = c["pcg_mgjac_info"]
        assert info["niter"] == int(ref[0]) and info["success"] == bool(ref[1])
        assert rel(x.toarray(), c["pcg_mgjac"]) <= 1e-8
        for m in (3, 1000):
            x, info = crl(A, b, tol=0.0 if m == 3 else 1e-5, maxiter=m)
            ref = c[f"crl_m{m}_info"]
            _check_crl(info, ref, x.toarray(), c[f"crl_m{m}"], m, rhs)


def test_setitem_recipe_matches_spl_standin(gpu):
    """`populate_2d_matrix` (`sources/utils.py:18-26`) through the spl-style setters."""
    from oracle import spl_standin as S
    from poms_amd.stencil import StencilMatrix, StencilVectorSpace
    n1, n2, p1, p2 = 9, 7, 2, 1
    V = StencilVectorSpace([n1, n2], [p1, p2])
    A = StencilMatrix(V)
    Vs = S.StencilVectorSpace([n1, n2], [p1, p2])
    As = S.StencilMatrix(Vs, Vs)
    for k1 in range(-p1, p1 + 1):
        for k2 in range(-p2, p2 + 1):
            A[:, :, k1, k2] = 10. - abs(k1) - abs(k2)
            As[:, :, k1, k2] = 10. - abs(k1) - abs(k2)
    A.remove_spurious_entries()
    As.remove_spurious_entries()
    np.testing.assert_array_equal(A._data, As._data)
    x = np.random.default_rng(1).uniform(-1, 1, (n1, n2))
    xs = S.StencilVector(Vs)
    xs._data[p1:p1 + n1, p2:p2 + n2] = x
    assert rel(A.dot(V.zeros().from_numpy(x)).to_local_numpy(), As.dot(xs)._data[p1:p1 + n1, p2:p2 + n2]) <= 1e-14
    assert A[3, 2, -1, 1] == As[3, 2, -1, 1]
    A[3, 2, 0, 0] = 42.0                         # re-upload after a host-side change
    x1 = V.zeros().from_numpy(x)
    y = A.dot(x1).to_local_numpy()
    As[3, 2, 0, 0] = 42.0
    assert rel(y, As.dot(xs)._data[p1:p1 + n1, p2:p2 + n2]) <= 1e-14


@pytest.mark.parametrize("shape,pads,align", [((23, 31), (2, 3), False), ((40, 37), (3, 3), True),
                                              ((9, 11, 13), (1, 2, 1), False), ((12, 10, 19), (2, 2, 2), True)])
def test_random_stencil_epilogues(gpu, shape, pads, align):
    import torch
    from poms_amd.stencil import StencilMatrix, StencilVectorSpace
    rng = np.random.default_rng(sum(shape))
    V = StencilVectorSpace(list(shape), list(pads), align=align)
    A = StencilMatrix(V)
    A._data[...] = rng.uniform(-1, 1, A._data.shape)
    c = tuple(p for p in pads)
    inner = tuple(slice(p, p + n) for p, n in zip(pads, shape))
    A._data[inner + c] += 4.0 * np.prod([2 * p + 1 for p in pads]) ** 0.5   # safe diagonal
    A.remove_spurious_entries()
    data = A._data.copy()
    x, b = rng.uniform(-1, 1, shape), rng.uniform(-1, 1, shape)
    xv, bv = V.zeros().from_numpy(x), V.zeros().from_numpy(b)
    Ax = stencil_dot_ref(data, x, pads)
    diag = data[inner + c]
    assert rel(A.dot(xv).to_local_numpy(), Ax) <= 1e-14
    assert rel(A.residual(bv, xv).to_local_numpy(), b - Ax) <= 1e-14
    xo = V.empty()
    nrm = A.jacobi_sweep(bv, xv, xo, 2.0 / 3.0, want_norm=True)
    dr = (2.0 / 3.0) * (b - Ax) / diag
    assert rel(xo.to_local_numpy(), x + dr) <= 1e-14
    assert abs(nrm - float(np.sum(dr * dr))) <= 1e-12 * float(np.sum(dr * dr))
    d1 = V.empty()
    n1 = A.diag_scale(bv, d1, 0.5, want_norm=True)
    assert rel(d1.to_local_numpy(), 0.5 * b / diag) <= 1e-15
    assert abs(n1 - float(np.sum((0.5 * b / diag) ** 2))) <= 1e-12 * n1
    q = V.empty()
    pq = A.dot_inner(xv, q)
    assert abs(float(pq) - float(np.sum(x * Ax))) <= 1e-12 * abs(float(np.sum(x * Ax))) + 1e-12
    full = xo._data.cpu().numpy().copy()       # ghosts untouched (zero)
    full[tuple(slice(p, p + n) for p, n in zip(pads, shape))] = 0.0
    assert not np.any(full[..., :V.padded_shape[-1]])

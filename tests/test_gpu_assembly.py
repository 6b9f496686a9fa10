"""On-device quadrature assembly: the reference's assembly_2d
stencils (golden), variable coefficients against the oracle's restatement of the
reference element loop, 3D against the Kronecker-sum stencil, and a solve on a
variable-coefficient operator."""
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


def maxrel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def test_device_assembly_matches_assembly_2d_golden(gpu, golden_dir):
    from poms_amd.assembly import assemble_stencil
    from poms_amd.splines import make_open_knots
    from poms_amd.stencil import StencilVectorSpace
    for name, c in load(golden_dir, "assembly_2d.npz").items():
        p = int(c["p"])
        ne = [int(v) for v in c["ne"]]
        V = StencilVectorSpace([e + p for e in ne], [p, p])
        A = assemble_stencil(V, [make_open_knots(p, e + p) for e in ne])
        assert maxrel(A._data, c["stencil"]) <= 1e-13, name


@pytest.mark.parametrize("p,ne", [((2, 3), (6, 5)), ((3, 3), (8, 7))])
def test_device_assembly_variable_coefficients_2d(gpu, p, ne):
    from poms_amd.assembly import assemble_stencil, axis_tables
    from poms_amd.splines import make_open_knots
    from poms_amd.stencil import StencilVectorSpace
    T = [make_open_knots(pd, e + pd) for pd, e in zip(p, ne)]
    tabs = [axis_tables(t, pd) for t, pd in zip(T, p)]
    X, Y = np.meshgrid(*[t["points"].reshape(-1) for t in tabs], indexing="ij")
    a = 1.0 + 0.5 * np.sin(3 * X) * np.cos(2 * Y)
    c = 2.0 + X * Y
    V = StencilVectorSpace([e + pd for pd, e in zip(p, ne)], list(p))
    A = assemble_stencil(V, T, a=a, c=lambda x, y: 2.0 + x * y)
    ref = orc.assembly_varcoef(T, list(p), a=a, c=c)
    assert maxrel(A._data, ref) <= 1e-13
    # and the operator applies as a general stencil
    x = np.random.default_rng(0).uniform(-1, 1, V.npts)
    y = A.dot(V.zeros().from_numpy(x)).to_local_numpy()
    assert maxrel(y.reshape(-1), A.tosparse() @ x.reshape(-1)) <= 1e-13


def test_device_assembly_3d_constant_is_kron_sum(gpu):
    from poms_amd.assembly import assemble_stencil
    from poms_amd.splines import assemble_1d, make_open_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, ne = 2, 6
    n = ne + p
    T = make_open_knots(p, n)
    V = StencilVectorSpace([n] * 3, [p] * 3)
    A = assemble_stencil(V, [T] * 3)
    M, K = assemble_1d(T, p, canonical=False)
    Ak = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x = np.random.default_rng(1).uniform(-1, 1, (n,) * 3)
    xv = V.zeros().from_numpy(x)
    assert maxrel(A.dot(xv).to_local_numpy(), Ak.dot(xv).to_local_numpy()) <= 1e-13
    a = lambda x, y, z: 1.0 + x + 0.5 * y * z
    Av = assemble_stencil(V, [T] * 3, a=a, mass_coef=0.5)
    from poms_amd.assembly import axis_tables
    tabs = [axis_tables(T, p)] * 3
    G = np.meshgrid(*[t["points"].reshape(-1) for t in tabs], indexing="ij")
    ref = orc.assembly_varcoef([T] * 3, [p] * 3, a=a(*G), mass_coef=0.5)
    assert maxrel(Av._data, ref) <= 1e-13


def test_pcg_on_variable_coefficient_operator(gpu):
    """pcg + damped Jacobi on a device-assembled variable-coefficient operator
    == the oracle pcg on the same stencil (the solvers take any general stencil)."""
    from poms_amd.assembly import assemble_stencil
    from poms_amd.solvers import damped_jacobi, pcg
    from poms_amd.splines import make_open_knots
    from poms_amd.stencil import StencilVectorSpace
    p, ne = 3, 12
    n = ne + p
    T = make_open_knots(p, n)
    V = StencilVectorSpace([n, n], [p, p])
    A = assemble_stencil(V, [T, T], a=lambda x, y: 1.0 + 10.0 * x * y)
    Acsr = A.tosparse()
    D = Acsr.diagonal()
    b = np.ones(n * n)
    x, info = pcg(A, damped_jacobi, V.zeros().from_numpy(b.reshape(n, n)), tol=0.0, maxiter=4)
    apply = lambda v: Acsr @ v
    xr, ir = orc.pcg(apply, lambda r: orc.damped_jacobi(apply, D, r), b, tol=0.0, maxiter=4)
    assert info["niter"] == ir["niter"]
    assert np.linalg.norm(x.toarray() - xr) <= 1e-9 * np.linalg.norm(xr)

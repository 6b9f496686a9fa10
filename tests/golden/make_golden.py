#!/usr/bin/env python3
"""Generate the golden fixtures from the REFERENCE ITSELF (this container only).

Imports the reference's own Python (read-only, from /root/reference):
  * `pyccel/pyccel_functions.py`  -> kron_dot_pyccel_2d (the native Kron kernel)
  * `sources/utils.py`            -> populate_1d_matrix / kron_dot_ref
  * `sources/matrix_assembler.py` -> assembly_2d, assembly_1d
  * `sources/solvers.py`          -> pcg, damped_jacobi, jacobi, crl
  * `sources/multilevels.py`      -> knots_to_insert
  * `sources/kron_product.py`     -> kron_solve_serial / kron_solve_par / to_bnd
  * `pyccel/pyccel_functions.py`  -> kron_solve_serial_pyccel_2d, kron_solve_par_bnd_pyccel_2d/_3d
  * `sources/solvers.py`          -> pcg_glt (GLT post-smoother)
  * `sources/mg_jac.py`           -> the two-level V-cycle driver, run as a script
with ``oracle/spl_standin.py`` registered for the absent third-party ``spl``
and ``mpi4py`` modules.  Writes small ``.npz`` fixtures next to this script;
nothing of the reference's source is copied.  The GPU box never runs this.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import contextlib
import io
import runpy
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))

from oracle import spl_standin  # noqa: E402

spl_standin.install()
sys.path.insert(0, str(REF / "sources"))
sys.path.insert(0, str(REF / "pyccel"))

import pyccel_functions as ref_pf  # noqa: E402
import utils as ref_utils  # noqa: E402
import solvers as ref_solvers  # noqa: E402
import matrix_assembler as ref_asm  # noqa: E402
import multilevels as ref_ml  # noqa: E402
import importlib.util as _ilu  # noqa: E402

# `sources/kron_product.py` (both sources/ and pyccel/ have a kron_product module;
# `solvers.pcg_glt` imports the sources one by name, `sources/solvers.py:241`)
_spec = _ilu.spec_from_file_location("kron_product", REF / "sources" / "kron_product.py")
ref_kp = _ilu.module_from_spec(_spec)
sys.modules["kron_product"] = ref_kp
_spec.loader.exec_module(ref_kp)
# `to_bnd` uses `dia_matrix` without importing it (`sources/kron_product.py:177`):
# pin the undefined name to scipy's, which it evidently means.
import scipy.sparse as _sps  # noqa: E402
ref_kp.dia_matrix = _sps.dia_matrix

S = spl_standin


def band_of(M1d):
    """(n, 2p+1) band rows of a 1D stand-in StencilMatrix."""
    p = M1d.pads[0]
    n = M1d._domain.npts[0]
    return M1d._data[p:p + n, :].copy()


def golden_kron_dot():
    out = {}
    # (a) the test_kron_dot recipe: 8x4, p=(2,1), populate_1d_matrix(5/6), X = 1
    #     (`sources/tests/test_kron_dot.py:14-40,125-126`)
    n1, n2, p1, p2 = 8, 4, 2, 1
    V = S.StencilVectorSpace([n1, n2], [p1, p2], [False, False])
    V1 = S.StencilVectorSpace([n1], [p1], [False])
    V2 = S.StencilVectorSpace([n2], [p2], [False])
    X = S.StencilVector(V)
    A = S.StencilMatrix(V1, V1)
    B = S.StencilMatrix(V2, V2)
    ref_utils.populate_1d_matrix(A, 5.)
    ref_utils.populate_1d_matrix(B, 6.)
    ref_utils.populate_2d_vector(X)
    Ab, Bb = band_of(A), band_of(B)
    Y = np.zeros_like(X._data)
    ref_pf.kron_dot_pyccel_2d(np.array([0, 0]), np.array([n1 - 1, n2 - 1]), np.array([p1, p2]),
                              X._data, np.zeros_like(X._data), Y, Ab, Bb)
    Yref = ref_utils.kron_dot_ref(A, B, X)  # scipy.sparse.kron(A, B) @ X.toarray()
    out["recipe"] = dict(X=X._data, A=Ab, B=Bb, Y=Y, Y_kron_ref=Yref, starts=[0, 0], ends=[n1 - 1, n2 - 1],
                         pads=[p1, p2])
    # (b) seeded random inputs, full grids and interior sub-blocks with ghost data
    cases = [(16, 12, 1, 1), (20, 24, 2, 2), (33, 17, 3, 3), (40, 30, 5, 5), (24, 31, 2, 3), (64, 64, 3, 3)]
    for ci, (m1, m2, q1, q2) in enumerate(cases):
        rng = np.random.default_rng(ci)
        Ab = rng.uniform(-1, 1, (m1, 2 * q1 + 1))
        Bb = rng.uniform(-1, 1, (m2, 2 * q2 + 1))
        for name, (st, en) in {"full": ((0, 0), (m1 - 1, m2 - 1)),
                               "block": ((m1 // 4, m2 // 3), (m1 - 2, m2 - 3))}.items():
            shp = (en[0] - st[0] + 1 + 2 * q1, en[1] - st[1] + 1 + 2 * q2)
            Xd = rng.uniform(-1, 1, shp)
            if name == "full":   # zero ghosts: a whole non-periodic grid on one rank
                Xd[:q1] = 0; Xd[-q1:] = 0; Xd[:, :q2] = 0; Xd[:, -q2:] = 0
            Y = np.zeros(shp)
            ref_pf.kron_dot_pyccel_2d(np.array(st), np.array(en), np.array([q1, q2]), Xd, np.zeros(shp), Y, Ab, Bb)
            out[f"rand{ci}_{name}"] = dict(X=Xd, A=Ab, B=Bb, Y=Y, starts=list(st), ends=list(en), pads=[q1, q2])
    with open(HERE / "kron_dot_2d.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


def golden_assembly():
    out = {}
    for p, (ne1, ne2) in [(1, (4, 4)), (1, (16, 16)), (2, (6, 9)), (3, (8, 8)), (3, (5, 7))]:
        S1 = S.SplineSpace(p, grid=np.linspace(0., 1., ne1 + 1))
        S2 = S.SplineSpace(p, grid=np.linspace(0., 1., ne2 + 1))
        Vh = S.TensorFemSpace(S1, S2)
        M = ref_asm.assembly_2d(Vh)           # `sources/matrix_assembler.py:84-179`
        Mseq = ref_asm.assembly_2d_seq(Vh)    # :183-253
        m1 = ref_asm.assembly_1d(S1)          # :10-77 (returns the mass matrix only)
        out[f"p{p}_{ne1}x{ne2}"] = dict(stencil=M._data, stencil_seq=Mseq._data, mass1d=band_of(m1),
                                       p=p, ne=[ne1, ne2])
    with open(HERE / "assembly_2d.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return out


def _problem(p, ne):
    S1 = S.SplineSpace(p, grid=np.linspace(0., 1., ne + 1))
    Vh = S.TensorFemSpace(S1, S.SplineSpace(p, grid=np.linspace(0., 1., ne + 1)))
    A = ref_asm.assembly_2d(Vh)
    return Vh.vector_space, A


def golden_solvers():
    out = {}
    for p, ne in [(1, 4), (1, 16), (3, 8)]:
        V, A = _problem(p, ne)
        x0 = S.StencilVector(V)
        for i1 in range(V.npts[0]):
            for i2 in range(V.npts[1]):
                x0[i1, i2] = i1 + i2 + 1.       # `sources/tests/test_djac.py:54-56`
        b = A.dot(x0)
        ones = S.StencilVector(V)
        ones[:, :] = 1.0                         # `sources/mg_jac.py:59-61`
        for rhs_name, rhs in (("manuf", b), ("ones", ones)):
            key = f"p{p}_ne{ne}_{rhs_name}"
            res = {"b": rhs.toarray()}
            for m in (1, 3, 10):
                res[f"djac_m{m}_tol0"] = ref_solvers.damped_jacobi(A, rhs, tol=0.0, maxiter=m).toarray()
            res["djac_default"] = ref_solvers.damped_jacobi(A, rhs).toarray()
            res["jacobi"] = ref_solvers.jacobi(A, rhs).toarray()
            for m in (1, 2, 5):
                x, info = ref_solvers.pcg(A, ref_solvers.damped_jacobi, rhs, tol=0.0, maxiter=m)
                res[f"pcg_m{m}_tol0"] = x.toarray()
                res[f"pcg_m{m}_tol0_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
            x, info = ref_solvers.pcg(A, ref_solvers.damped_jacobi, rhs, tol=1e-6, maxiter=10)
            res["pcg_mgjac"] = x.toarray()
            res["pcg_mgjac_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
            for m, tl in ((3, 0.0), (1000, 1e-5)):      # conjugate residual, `sources/solvers.py:3-65`
                x, info = ref_solvers.crl(A, rhs, tol=tl, maxiter=m)
                res[f"crl_m{m}"] = x.toarray()
                res[f"crl_m{m}_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
            res["p"], res["ne"] = p, ne
            out[key] = res
    with open(HERE / "solvers_2d.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


def golden_knots():
    out = {}
    for p, nc, nf in [(1, 8, 10), (3, 8, 13), (3, 8, 12), (2, 8, 16), (3, 11, 19)]:
        Tc, Tf = S.make_open_knots(p, nc), S.make_open_knots(p, nf)
        out[f"p{p}_nc{nc}_nf{nf}"] = dict(Tc=Tc, Tf=Tf, ts=ref_ml.knots_to_insert(Tf, nf, p, Tc, nc, p))
    with open(HERE / "knots_to_insert.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


def golden_vcycle():
    """Run `sources/mg_jac.py` itself (as __main__) with p, nf on argv."""
    # the driver imports names that do not exist (`sources/mg_jac.py:13`):
    # pin them to the functions they were evidently meant to be.
    ref_asm.assembly = ref_asm.assembly_2d
    ref_asm.assembly_seq = ref_asm.assembly_2d_seq
    out = {}
    for p, nf in [(1, 10), (2, 12), (3, 13)]:
        argv = sys.argv
        sys.argv = ["mg_jac.py", str(p), str(nf)]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                g = runpy.run_path(str(REF / "sources" / "mg_jac.py"), run_name="__main__")
        finally:
            sys.argv = argv
        out[f"p{p}_nf{nf}"] = dict(
            xf2=g["xf_2"].toarray(), xf_pre=g["xf"].toarray(), T=np.asarray(g["T"]), Tc=g["Tc"], Tf=g["Tf"],
            Ts=g["Ts"], P1=g["P1"].toarray(),
            info_pre=[g["info_pre"]["niter"], float(g["info_pre"]["success"]), g["info_pre"]["res_norm"]],
            info_pos=[g["info_pos"]["niter"], float(g["info_pos"]["success"]), g["info_pos"]["res_norm"]],
            p=p, nf=nf, nc=8)
    with open(HERE / "vcycle_mg_jac.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


class _Dense:
    """Minimal object with ``toarray()`` (what `to_bnd` and `kron_solve_*` call)."""

    def __init__(self, a):
        self.a = np.asarray(a, dtype=np.float64)

    def toarray(self):
        return self.a.copy()


def _recipe_band(n, p, lo, di, up):
    """Dense n x n with `lo` on sub-diagonals 1..p, `di` on the diagonal, `up` on
    super-diagonals 1..p -- the StencilMatrix slice fills of
    `pyccel/test_kron_solve.py:130-141,226-244` (after remove_spurious_entries)."""
    A = np.zeros((n, n))
    for i in range(n):
        for k in range(-p, p + 1):
            if 0 <= i + k < n:
                A[i, i + k] = di if k == 0 else (lo if k < 0 else up)
    return A


def _populate(n, p, diag):
    """`sources/utils.py:6-15` populate_1d_matrix as a dense matrix (M[i,k] = k, M[i,0] = diag)."""
    A = np.zeros((n, n))
    for i in range(n):
        for k in range(-p, p + 1):
            if 0 <= i + k < n:
                A[i, i + k] = diag if k == 0 else k
    return A


def _subcoms(nd):
    return [S._SubComm() for _ in range(nd)]


def golden_kron_solve():
    import scipy.linalg as sla
    out = {}
    # (a) test_par_banded_2d recipe (`pyccel/test_kron_solve.py:117-160`) through the
    #     native band kernel and the dense serial kernel
    cases2 = [("banded", 8, 6, 1, 1), ("banded", 10, 12, 2, 3), ("banded", 16, 16, 3, 3),
              ("populate", 12, 9, 2, 1), ("populate", 10, 10, 3, 3), ("random", 20, 17, 2, 3)]
    for ci, (kind, n1, n2, p1, p2) in enumerate(cases2):
        if kind == "banded":
            A1, A2 = _recipe_band(n1, p1, -4, 10 * p1, -2), _recipe_band(n2, p2, -1, 2 * p2, -2)
            Yg = np.array([[(i1 + 1) * 10 + (i2 + 1) for i2 in range(n2)] for i1 in range(n1)], dtype=float)
        elif kind == "populate":     # `sources/tests/test_kron_solve.py` test_ser: diag 5 / 6, Y = 1
            A1, A2 = _populate(n1, p1, 5.0), _populate(n2, p2, 6.0)
            Yg = np.ones((n1, n2))
        else:
            rng = np.random.default_rng(100 + ci)
            A1 = _recipe_band(n1, p1, 0, 0, 0) + np.triu(np.tril(rng.uniform(-1, 1, (n1, n1)), p1), -p1)
            A2 = np.triu(np.tril(rng.uniform(-1, 1, (n2, n2)), p2), -p2)
            Yg = rng.uniform(-1, 1, (n1, n2))
        Y = np.zeros((n1 + 2 * p1, n2 + 2 * p2))
        Y[p1:p1 + n1, p2:p2 + n2] = Yg
        A1b, la1, ua1 = ref_kp.to_bnd(_Dense(A1))
        A2b, la2, ua2 = ref_kp.to_bnd(_Dense(A2))
        X = np.zeros_like(Y)
        ref_pf.kron_solve_par_bnd_pyccel_2d(np.asfortranarray(A1b), la1, ua1, np.asfortranarray(A2b), la2, ua2,
                                            X, Y, np.array([n1, n2]), np.array([p1, p2]), np.array([0, 0]),
                                            np.array([n1 - 1, n2 - 1]), _subcoms(2), n1, 0, n2, 0)
        Xs = np.zeros_like(Y)
        ref_pf.kron_solve_serial_pyccel_2d(np.asfortranarray(A1), np.asfortranarray(A2), Xs, Y,
                                           np.array([n1, n2]), np.array([p1, p2]))
        Xk = sla.solve(np.kron(A1, A2), Yg.reshape(-1)).reshape(n1, n2)   # kron_solve_seq_ref_2d
        out[f"d2_{kind}_{n1}x{n2}_p{p1}{p2}"] = dict(A1=A1, A2=A2, Y=Y, X_bnd=X, X_serial=Xs, X_kron_ref=Xk,
                                                     points=[n1, n2], pads=[p1, p2])
    # (b) the spl-level wrappers `sources/kron_product.py:93-158` on stand-in vectors
    n1, n2, p1, p2 = 9, 7, 2, 2
    V = S.StencilVectorSpace([n1, n2], [p1, p2], [False, False])
    Yv = S.StencilVector(V)
    ref_utils.populate_2d_vector(Yv)
    A1, A2 = _populate(n1, p1, 5.0), _populate(n2, p2, 6.0)
    out["spl_wrappers"] = dict(A1=A1, A2=A2, Y=Yv._data.copy(),
                               X_serial=ref_kp.kron_solve_serial(_Dense(A1), _Dense(A2), Yv)._data,
                               X_par=ref_kp.kron_solve_par(_Dense(A1), _Dense(A2), Yv)._data,
                               points=[n1, n2], pads=[p1, p2])
    # (c) 3D recipe (`pyccel/test_kron_solve.py:196-262`)
    for (n1, n2, n3, p1, p2, p3) in [(6, 5, 7, 1, 1, 1), (8, 9, 10, 2, 3, 2)]:
        A1 = _recipe_band(n1, p1, -4, 10 * p1, -4)
        A2 = _recipe_band(n2, p2, -1, 2 * p2, -1)
        A3 = _recipe_band(n3, p3, -2, 3 * p2, -2)
        Yg = np.array([[[(i1 + 1) * 100 + (i2 + 1) * 10 + (i3 + 1) for i3 in range(n3)] for i2 in range(n2)]
                       for i1 in range(n1)], dtype=float)
        Y = np.zeros((n1 + 2 * p1, n2 + 2 * p2, n3 + 2 * p3))
        Y[p1:p1 + n1, p2:p2 + n2, p3:p3 + n3] = Yg
        bands = [ref_kp.to_bnd(_Dense(A)) for A in (A1, A2, A3)]
        X = np.zeros_like(Y)
        args = []
        for b, l, u in bands:
            args += [np.asfortranarray(b), l, u]
        ref_pf.kron_solve_par_bnd_pyccel_3d(*args, X, Y, np.array([n1, n2, n3]), np.array([p1, p2, p3]),
                                            np.array([0, 0, 0]), np.array([n1 - 1, n2 - 1, n3 - 1]), _subcoms(3),
                                            n1, 0, n2, 0, n3, 0)
        Xk = sla.solve(np.kron(np.kron(A1, A2), A3), Yg.reshape(-1)).reshape(n1, n2, n3)
        out[f"d3_{n1}x{n2}x{n3}_p{p1}{p2}{p3}"] = dict(A1=A1, A2=A2, A3=A3, Y=Y, X_bnd=X, X_kron_ref=Xk,
                                                        points=[n1, n2, n3], pads=[p1, p2, p3])
    with open(HERE / "kron_solve.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


def golden_pcg_glt():
    """`sources/solvers.py:239-306` with the preconditioner matrices M1, M2 given as
    band matrices of the (restated, unpinned) cardinal-spline collocation matrix."""
    from oracle.poms_oracle import collocation_cardinal_splines
    out = {}
    for p, ne in [(1, 4), (2, 8), (3, 8), (3, 12)]:
        V, A = _problem(p, ne)
        n1, n2 = V.npts
        x0 = S.StencilVector(V)
        for i1 in range(n1):
            for i2 in range(n2):
                x0[i1, i2] = i1 + i2 + 1.          # `sources/tests/test_glt.py:53-56`
        b = A.dot(x0)
        M1 = _Dense(collocation_cardinal_splines(p, n1))
        M2 = _Dense(collocation_cardinal_splines(p, n2))
        res = {"b": b.toarray(), "M1": M1.a, "M2": M2.a, "p": p, "ne": ne}
        x, info = ref_solvers.pcg_glt(A, M1, M2, b, tol=1e-8, maxiter=100)   # test_glt.py:70
        res["glt_test"] = x.toarray()
        res["glt_test_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
        for m in (1, 3):
            x, info = ref_solvers.pcg_glt(A, M1, M2, b, tol=0.0, maxiter=m)
            res[f"glt_m{m}_tol0"] = x.toarray()
            res[f"glt_m{m}_tol0_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
        ones = S.StencilVector(V)
        ones[:, :] = 1.0
        xs = S.StencilVector(V)
        for i1 in range(n1):
            for i2 in range(n2):
                xs[i1, i2] = 0.01 * (i1 - i2)
        x, info = ref_solvers.pcg_glt(A, M1, M2, ones, x0=xs, tol=1e-6, maxiter=p + 1)   # mg_glt.py:123
        res["glt_post"] = x.toarray()
        res["glt_post_x0"] = xs.toarray()
        res["glt_post_info"] = [info["niter"], float(info["success"]), info["res_norm"]]
        out[f"p{p}_ne{ne}"] = res
    with open(HERE / "pcg_glt.npz", "wb") as f:
        np.savez_compressed(f, **{f"{k}__{kk}": np.asarray(vv) for k, v in out.items() for kk, vv in v.items()})
    return len(out)


if __name__ == "__main__":
    print("kron_dot cases:", golden_kron_dot())
    print("assembly cases:", len(golden_assembly()))
    print("knots cases:", golden_knots())
    print("solver cases:", golden_solvers())
    print("vcycle cases:", golden_vcycle())
    print("kron solve cases:", golden_kron_solve())
    print("pcg_glt cases:", golden_pcg_glt())

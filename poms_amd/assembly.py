"""On-device quadrature assembly of B-spline stencil operators.

The reference assembles ``-Δu + u`` element by element in Python
(`sources/matrix_assembler.py:84-179`, ``assembly_2d``: 222 s on one process for
the slides' grid, `sources/scalability.py:10`).  Here the host builds only the 1D
tables of each axis -- elements (non-empty knot spans), Gauss points and weights,
the ``p+1`` local B-splines and their derivatives at those points (Cox-de Boor,
:func:`poms_amd.splines.basis_funs_ders`) -- and ``poms_op_assemble_stencil``
forms every stencil coefficient on the device, one thread per (row, offset):

    M[i, j] = Σ_e Σ_q w_q (c(x_q) φ_i φ_j + a(x_q) ∇φ_i·∇φ_j)

With ``a = c = 1`` this is ``assembly_2d``'s operator (pinned by its golden
stencils); variable ``a``/``c`` (callables on the quadrature grid, or arrays of
its shape) give operators that are not Kronecker sums, applied by the
general-stencil kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .splines import basis_funs_ders
from .stencil import StencilMatrix, StencilVectorSpace


def axis_tables(T: np.ndarray, p: int, nquad: int | None = None) -> dict:
    """1D element tables of knot vector ``T`` (degree ``p``, ``nquad`` Gauss points,
    default ``p+1`` -- the reference's ``quad_order``)."""
    T = np.asarray(T, dtype=np.float64)
    n = len(T) - p - 1
    nq = p + 1 if nquad is None else int(nquad)
    xg, wg = np.polynomial.legendre.leggauss(nq)
    spans = [s for s in range(p, n) if T[s + 1] > T[s]]
    nel = len(spans)
    basis = np.zeros((nel, nq, p + 1, 2))
    weights = np.zeros((nel, nq))
    points = np.zeros((nel, nq))
    first = np.array([s - p for s in spans], dtype=np.int32)
    for e, s in enumerate(spans):
        a, b = T[s], T[s + 1]
        half = 0.5 * (b - a)
        for g in range(nq):
            x = a + half * (xg[g] + 1.0)
            points[e, g] = x
            weights[e, g] = half * wg[g]
            D = basis_funs_ders(T, p, x, s, 1)
            basis[e, g, :, 0] = D[0]
            basis[e, g, :, 1] = D[1]
    es = np.full(n, nel, dtype=np.int32)
    ee = np.full(n, -1, dtype=np.int32)
    for e, f in enumerate(first):
        for i in range(f, f + p + 1):
            es[i] = min(es[i], e)
            ee[i] = max(ee[i], e)
    return dict(n=n, p=p, nel=nel, nq=nq, first=first, es=es, ee=ee, basis=basis, weights=weights, points=points)


def _coef_field(f, tabs, device):
    if f is None:
        return None
    if callable(f):
        grids = np.meshgrid(*[t["points"].reshape(-1) for t in tabs], indexing="ij")
        vals = np.asarray(f(*grids), dtype=np.float64)
    else:
        vals = np.asarray(f, dtype=np.float64)
    shape = tuple(t["nel"] * t["nq"] for t in tabs)
    vals = np.broadcast_to(vals, shape)
    return torch.from_numpy(np.array(vals, dtype=np.float64, order="C")).to(device)


def assemble_stencil(V: StencilVectorSpace, knots, a=None, c=None, mass_coef: float = 1.0,
                     nquad: int | None = None) -> StencilMatrix:
    """``-∇·(a ∇u) + c u`` on the tensor space of ``knots`` (one knot vector per axis,
    degree = the space's pads), assembled on the device.  ``a``/``c``: None (1 and
    ``mass_coef``), a callable of the quadrature-point coordinates (``meshgrid``,
    ``indexing='ij'``) or an array of the quadrature grid's shape."""
    nd = V.ndim
    if len(knots) != nd:
        raise ValueError(f"{nd}D space needs {nd} knot vectors")
    tabs = [axis_tables(np.asarray(T, float), V.pads[d], nquad) for d, T in enumerate(knots)]
    for d, t in enumerate(tabs):
        if t["n"] != V.npts[d]:
            raise ValueError(f"axis {d}: knots give {t['n']} basis functions, space has {V.npts[d]}")
    lead = 3 - nd
    keep = []

    def arr3(key, ctype, np_dtype):
        out = (C.c_void_p * 3)()
        for k, t in enumerate(tabs):
            a_ = np.ascontiguousarray(t[key], dtype=np_dtype)
            keep.append(a_)
            out[lead + k] = a_.ctypes.data
        return out

    ints = lambda key: [0] * lead + [int(t[key]) for t in tabs]
    nel = (C.c_int * 3)(*ints("nel"))
    nq = (C.c_int * 3)(*ints("nq"))
    pp = (C.c_int * 3)(*ints("p"))
    nglob = (C.c_int64 * 3)(*([1] * lead + [int(t["n"]) for t in tabs]))
    dev = f"cuda:{V.device}"
    aq, cq = _coef_field(a, tabs, dev), _coef_field(c, tabs, dev)
    h = C.c_void_p()
    _lib.call("poms_op_assemble_stencil", V.ctx, nd, C.byref(V.layout), nel, nq, pp,
              arr3("first", C.c_int, np.int32), arr3("es", C.c_int, np.int32), arr3("ee", C.c_int, np.int32),
              arr3("basis", C.c_double, np.float64), arr3("weights", C.c_double, np.float64), nglob,
              None if aq is None else C.c_void_p(aq.data_ptr()), None if cq is None else C.c_void_p(cq.data_ptr()),
              float(mass_coef), int(V.starts[0]) if nd == 3 else 0, C.byref(h))
    return StencilMatrix._from_handle(V, h)

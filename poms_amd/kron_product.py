"""Kronecker mat-vec entry points with the reference's names and conventions.

* :func:`kron_dot_v2` ``(A, B, X) -> Y = (A⊗B) X`` on a 2D
  :class:`~poms_amd.stencil.StencilVector` (`sources/kron_product.py:56-89`):
  ghost exchange of X, fused two-pass apply on the GPU, fresh result vector.
  3D: ``kron_dot_3d(A, B, C, X)``.
* :func:`kron_dot_pyccel_2d` ``(starts, ends, pads, X, X_tmp, Y, A, B)`` --
  the native kernel's signature (`pyccel/pyccel_functions.py:3-21`) on host
  NumPy arrays, writing ``Y`` in place, through ``poms_kron_dot_2d``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from . import runtime as rt
from .stencil import KronOperator, StencilVector

_CACHE: dict = {}


def _op_for(V, factors):
    key = (id(V), tuple(id(f) for f in factors))
    ent = _CACHE.get(key)
    bands = [getattr(f, "band", f) for f in factors]
    if ent is not None and all(np.array_equal(a, b) for a, b in zip(ent[1], bands)):
        return ent[0]
    op = KronOperator.product(V, factors)
    _CACHE.clear()  # keep at most one cached operator alive
    _CACHE[key] = (op, [np.array(b, copy=True) for b in bands])
    return op


def kron_dot_v2(A, B, X: StencilVector) -> StencilVector:
    """``Y = (A ⊗ B) X`` (A acts on axis 0, B on axis 1)."""
    if X.space.ndim != 2:
        raise ValueError("kron_dot_v2 is the 2D product; use kron_dot_3d for 3D")
    return _op_for(X.space, (A, B)).dot(X)


def kron_dot_3d(A, B, Cf, X: StencilVector) -> StencilVector:
    if X.space.ndim != 3:
        raise ValueError("kron_dot_3d needs a 3D vector")
    return _op_for(X.space, (A, B, Cf)).dot(X)


def kron_dot_pyccel_2d(starts, ends, pads, X, X_tmp, Y, A, B):
    """Host-array drop-in of the pyccel kernel; updates ``Y`` in place and returns it."""
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    ends = np.ascontiguousarray(ends, dtype=np.int64)
    pads = np.ascontiguousarray(pads, dtype=np.int64)
    for name, arr in (("X", X), ("Y", Y), ("A", A), ("B", B)):
        if not (isinstance(arr, np.ndarray) and arr.dtype == np.float64 and arr.flags.c_contiguous):
            raise TypeError(f"{name} must be a C-contiguous float64 numpy array")
    shape = (int(ends[0] - starts[0] + 1 + 2 * pads[0]), int(ends[1] - starts[1] + 1 + 2 * pads[1]))
    if X.shape != shape or Y.shape != shape:
        raise ValueError(f"X/Y must have the padded local shape {shape}")
    if A.shape[1] != 2 * pads[0] + 1 or B.shape[1] != 2 * pads[1] + 1:
        raise ValueError("A/B band width must be 2p+1")
    ctx = rt.ctx(rt.device_index())
    xt = X_tmp.ctypes.data_as(C.c_void_p) if isinstance(X_tmp, np.ndarray) else None
    _lib.call("poms_kron_dot_2d", ctx, starts.ctypes.data_as(C.c_void_p), ends.ctypes.data_as(C.c_void_p),
              pads.ctypes.data_as(C.c_void_p), X.ctypes.data_as(C.c_void_p), xt, Y.ctypes.data_as(C.c_void_p),
              A.ctypes.data_as(C.c_void_p), A.shape[0], B.ctypes.data_as(C.c_void_p), B.shape[0])
    return Y

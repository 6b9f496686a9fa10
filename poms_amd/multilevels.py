"""Knot-insertion multilevel set-up and the device transfer operators.

* :func:`knots_to_insert` -- interior knots of the fine knot vector that are
  absent from the coarse one, same loop and float comparisons as
  `sources/multilevels.py:7-33`.
* :class:`KronTransfer` -- ``R = (P0⊗P1⊗P2)^T`` and ``P = P0⊗P1⊗P2`` applied
  by sum-factorised device passes (``poms_restrict`` / ``poms_prolong_add``),
  replacing the materialised ``scipy.sparse.kron`` products of
  `sources/mg_jac.py:67-70,94,102`.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np
import torch

from . import _lib
from . import runtime as rt
from .stencil import StencilVector, StencilVectorSpace, F64


def knots_to_insert(Tf, nf, pf, Tc, nc, pc):
    """Knots of ``Tf`` (interior) not present in ``Tc`` (`sources/multilevels.py:7-33`).

    The reference scans ``Tc[pc+1], Tc[pc+2], ...`` until the first knot larger
    than ``t`` or past index ``nc`` and inserts ``t`` when no exact match was
    seen; on a sorted knot vector that is exact-equality membership in
    ``Tc[pc+1 .. nc]``.  Multiplicities are ignored exactly as there.
    """
    Tf = np.asarray(Tf, dtype=np.float64)
    Tc = np.asarray(Tc, dtype=np.float64)
    cand = Tf[pf + 1:nf]
    present = np.isin(cand, Tc[pc + 1:nc + 1])
    return np.ascontiguousarray(cand[~present])


class KronTransfer:
    """Restriction / prolongation between a fine :class:`StencilVectorSpace`
    (possibly a slab or a Cart block) and a dense, replicated coarse vector of ``prod(nc)`` doubles."""

    def __init__(self, V: StencilVectorSpace, P: Sequence[np.ndarray]):
        nd = V.ndim
        if len(P) != nd:
            raise ValueError("need one 1D prolongation factor per axis")
        self.space = V
        self.P = [np.ascontiguousarray(p, dtype=np.float64) for p in P]
        for d, p in enumerate(self.P):
            if p.shape[0] != V.npts[d]:
                raise ValueError(f"axis {d}: P has {p.shape[0]} rows, space has {V.npts[d]} points")
        self.nc = tuple(p.shape[1] for p in self.P)
        lead = 3 - nd
        # rows of this rank: axis 0 of a 3D space whole (global offset g0), the other
        # axes of a Cart block sliced to the owned rows
        Pl = list(self.P)
        nfl = list(V.npts)
        if V.is_cart:
            for d in range(1 if nd == 3 else 0, nd):
                Pl[d] = np.ascontiguousarray(self.P[d][V.starts[d]:V.ends[d] + 1])
                nfl[d] = Pl[d].shape[0]
        nf3 = (1,) * lead + tuple(nfl)
        nc3 = (1,) * lead + self.nc
        ones = np.ones((1, 1))
        P3 = [ones] * lead + Pl
        self._keep = P3
        nf_arr = (C.c_int64 * 3)(*nf3)
        nc_arr = (C.c_int64 * 3)(*nc3)
        parr = (C.c_void_p * 3)(*[p.ctypes.data_as(C.c_void_p) for p in P3])
        self._h = C.c_void_p()
        _lib.call("poms_transfer_create", V.ctx, 3 if nd == 3 else 2, C.byref(V.layout),
                  V.starts[0] if nd == 3 else 0, nf_arr, nc_arr, parr, C.byref(self._h))
        self.ncoarse = int(np.prod(self.nc))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib.poms_transfer_destroy(h)
            except Exception:
                pass
            self._h = None

    def coarse_empty(self) -> torch.Tensor:
        return torch.empty(self.ncoarse, dtype=F64, device=f"cuda:{self.space.device}")

    def restrict(self, fine: StencilVector, out: torch.Tensor | None = None, allreduce: bool = True) -> torch.Tensor:
        """``rc = R rf`` (+ sum over slabs, `sources/mg_jac.py:94-95`)."""
        out = self.coarse_empty() if out is None else out
        _lib.call("poms_restrict", self._h, rt.ptr(fine._data), rt.ptr(out), rt.stream_handle())
        if allreduce and self.space.is_distributed:
            d = self.space.dist
            if d.native is not None:   # the library's communicator, on the device stream
                d.native.allreduce(out, rt.stream_handle(), wait_back=True)
            else:
                rt.Comm.from_env(d.group).allreduce_sum_(out)
        return out

    def set_operator(self, A) -> bool:
        """Prepare the fused ``R (b - A x)`` for the Kronecker operator ``A`` (a
        :class:`~poms_amd.stencil.KronOperator` on this transfer's space): the host forms
        ``G = F^T P_d`` for every 1D factor ``F`` of ``A`` (rows sliced like ``P_d``).
        Returns False where the fused path does not apply (banded transfers, coarse
        extents > 32; general stencils), and the caller keeps residual + restrict."""
        from .splines import band_to_dense
        V = self.space
        if A.space is not V or A.form not in ("sum", "single") or max(self.nc) > 32:
            return False
        nd = V.ndim
        lead = 3 - nd
        P = A.pmax

        def dense(band):   # 1-row bands are the scalar factors of the 1D operator
            return band[:, P:P + 1].copy() if band.shape[0] == 1 else band_to_dense(band)

        # role -> storage axis (poms_op_create's factor order)
        roles = ["A0", "M0", "A1", "B1", "M2", "K2"] if A.form == "sum" else ["F0", None, "F1", None, "F2", None]
        Pl = [np.ones((1, 1))] * lead + list(self.P)
        G = []
        for r, name in enumerate(roles):
            ax = r // 2
            if name is None or (ax == 0 and nd < 3):
                G.append(None)
                continue
            g = dense(A.bands[name]).T @ Pl[ax]
            if V.is_cart and ax >= 1 and g.shape[0] > 1:   # (KronTransfer's own slicing of P)
                d = ax - lead
                g = g[V.starts[d]:V.ends[d] + 1]
            G.append(np.ascontiguousarray(g, dtype=np.float64))
        self._G = G
        garr = (C.c_void_p * 6)(*[None if g is None else g.ctypes.data_as(C.c_void_p) for g in G])
        try:
            _lib.call("poms_transfer_set_operator", self._h, _lib.FORM_SUM if A.form == "sum" else _lib.FORM_SINGLE,
                      garr)
        except _lib.PomsError:
            return False
        self._op = A
        return True

    def resid_restrict(self, A, b: StencilVector, x: StencilVector, out: torch.Tensor | None = None,
                       allreduce: bool = True) -> torch.Tensor:
        """``rc = R (b - A x)`` (+ sum over slabs) without storing the residual
        (`sources/mg_jac.py:93-95`; fused: one pass over x and b instead of the residual's
        24 B/DOF plus the restriction's 8)."""
        if getattr(self, "_op", None) is not A and not self.set_operator(A):
            raise ValueError("fused residual -> restriction does not apply to this operator / transfer")
        out = self.coarse_empty() if out is None else out
        _lib.call("poms_resid_restrict", self._h, rt.ptr(b._data), rt.ptr(x._data), rt.ptr(out), rt.stream_handle())
        if allreduce and self.space.is_distributed:
            d = self.space.dist
            if d.native is not None:
                d.native.allreduce(out, rt.stream_handle(), wait_back=True)
            else:
                rt.Comm.from_env(d.group).allreduce_sum_(out)
        return out

    def prolong_add(self, coarse: torch.Tensor, fine: StencilVector) -> StencilVector:
        """``fine += P xc`` on the owned slab (`sources/mg_jac.py:102-112`)."""
        _lib.call("poms_prolong_add", self._h, rt.ptr(coarse), rt.ptr(fine._data), rt.stream_handle())
        fine._mark_written()
        return fine

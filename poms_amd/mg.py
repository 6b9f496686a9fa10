"""Two-level B-spline multigrid V-cycle (`sources/mg_jac.py`), on the device.

Set-up (host, once) follows `sources/mg_jac.py:25-81`:
coarse knots ``Tc``, fine knots ``Tf``, inserted knots
``Ts = knots_to_insert(Tf, nf, p, Tc, nc, p)``, fine space on
``T = sort(Tc ∪ Ts)``, operator ``-Δu + u``, ``P1 = matrix_multi_stages(Ts,
nc, p, Tc)``, ``R1 = P1^T``, Galerkin ``Ac = R Af P``.  Because every factor
is a Kronecker product, ``Ac = Σ_t ⊗_d (P1^T F_{t,d} P1)`` exactly; it is
factorised on the host (the reference's ``splu``) and its inverse applied on
the device.

Cycle (`sources/mg_jac.py:84-119`):
    xf, info_pre = pcg(Af, damped_jacobi, bf, tol, maxiter)     # pre-smoothing
    rc = R (bf - Af xf) (+ all-reduce over slabs)                 # residual -> restriction, fused
    xc = Ac^{-1} rc                                               # coarse solve
    xf = xf + P xc ; ghost exchange                               # correction
    xf2, info_pos = pcg(Af, damped_jacobi, bf, x0=xf, tol, maxiter)  # post-smoothing

``post_smoother="glt"`` runs `sources/mg_glt.py:113-123` instead: the post-smoother
is ``pcg_glt(Af, M1, M2, bf, x0=xf, tol, maxiter=p+1)``, preconditioned by the
Kronecker direct solve with the cardinal-spline collocation matrices
(``collocation_cardinal_splines(p, n)`` per axis, `sources/mg_glt.py:115-118`).

Grid convention: ``ncells_fine`` / ``ncells_coarse`` count CELLS; the knot
vectors have ``n = N + p`` basis functions.  (The reference passes ``nc = 8``
as a number of basis functions to ``make_open_knots``; with a uniform fine
grid of 512 cells that would make the union knot vector non-uniform, so the
benchmark nests an 8-cell coarse grid instead.  Both conventions are
supported through ``knots_coarse`` / ``knots_fine``.)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import scipy.linalg as sla
import torch

from . import _lib
from . import runtime as rt
from .multilevels import KronTransfer, knots_to_insert
from .solvers import damped_jacobi, pcg
from .splines import assemble_1d, matrix_multi_stages, uniform_knots
from .stencil import F64, KronOperator, StencilVector, StencilVectorSpace


def two_level_setup_1d(p: int, Tf: np.ndarray, Tc: np.ndarray):
    """1D pieces of the two-level hierarchy: fine knots T, inserted knots Ts, P1 (nf x nc)."""
    nf = len(Tf) - p - 1
    nc = len(Tc) - p - 1
    Ts = knots_to_insert(Tf, nf, p, Tc, nc, p)
    T = np.sort(np.concatenate([Tc, Ts]))
    P1 = matrix_multi_stages(Ts, nc, p, Tc)
    return T, Ts, P1


def galerkin_coarse_dense(Mc: np.ndarray, Kc: np.ndarray, ndim: int, mass_coef: float = 1.0) -> np.ndarray:
    """Dense ``Ac = c Mc⊗Mc(⊗Mc) + Σ_d (Kc on axis d, Mc elsewhere)``."""
    def kr(ms):
        out = ms[0]
        for m in ms[1:]:
            out = np.kron(out, m)
        return out

    A = mass_coef * kr([Mc] * ndim)
    for d in range(ndim):
        A = A + kr([Kc if e == d else Mc for e in range(ndim)])
    return A


class TwoLevelVCycle:
    """Two-level V-cycle on an ``ndim``-D tensor B-spline space of degree ``p``."""

    def __init__(self, p: int, ncells_fine: int, ncells_coarse: int = 8, ndim: int = 3, *,
                 dist=None, mass_coef: float = 1.0, device=None, knots_fine=None, knots_coarse=None,
                 tol: float = 1e-6, maxiter: int = 10, chunk: int = 0, align: bool = True,
                 post_smoother: str = "jacobi", fused_restrict: bool | None = None):
        self.p, self.ndim = int(p), int(ndim)
        if post_smoother not in ("jacobi", "glt"):
            raise ValueError("post_smoother must be 'jacobi' (mg_jac.py) or 'glt' (mg_glt.py)")
        self.post_smoother = post_smoother
        Tc = uniform_knots(p, ncells_coarse) if knots_coarse is None else np.asarray(knots_coarse, float)
        Tf = uniform_knots(p, ncells_fine) if knots_fine is None else np.asarray(knots_fine, float)
        T, Ts, P1 = two_level_setup_1d(p, Tf, Tc)
        self.Tc, self.Tf, self.T, self.Ts, self.P1 = Tc, Tf, T, Ts, P1
        n = len(T) - p - 1
        self.n = n
        M, K = assemble_1d(T, p)
        self.M1d, self.K1d = M, K
        # line-aligned rows (pitch a multiple of 16 doubles): the v5 operator kernel
        # then stores whole 128-B lines only
        self.space = StencilVectorSpace([n] * ndim, [p] * ndim, dist=dist, device=device, align=align)
        self.A = KronOperator.laplace(self.space, [M] * ndim, [K] * ndim, mass_coef=mass_coef)
        if chunk:
            self.A.set_chunk(chunk)
        self.transfer = KronTransfer(self.space, [P1] * ndim)
        # residual -> restriction in one pass over x and b (KronTransfer.resid_restrict);
        # False: the residual vector and the restriction, as the reference computes them.
        # None: fused in 3D (515^3: 0.70 ms against 0.92 for the pair), not in 2D, where
        # the passes are latency-bound (1027^2: 44.8 against 42.5 us)
        if fused_restrict is None:   # (POMS_FUSED_RESTRICT: 0 never, all in every dimension)
            fr = os.environ.get("POMS_FUSED_RESTRICT", "1")
            fused_restrict = fr == "all" or (ndim == 3 and fr != "0")
        self.fused_restrict = bool(fused_restrict) and self.transfer.set_operator(self.A)
        from .splines import band_to_dense
        Md, Kd = band_to_dense(M), band_to_dense(K)
        Mc, Kc = P1.T @ Md @ P1, P1.T @ Kd @ P1
        Ac = galerkin_coarse_dense(Mc, Kc, ndim, mass_coef)
        self.Ac = Ac
        lu = sla.lu_factor(Ac)
        Ainv = sla.lu_solve(lu, np.eye(Ac.shape[0]))
        dev = f"cuda:{self.space.device}"
        self.Ainv = torch.from_numpy(np.ascontiguousarray(Ainv)).to(dev)
        self.rc = torch.empty(Ac.shape[0], dtype=F64, device=dev)
        self.xc = torch.empty(Ac.shape[0], dtype=F64, device=dev)
        self.tol, self.maxiter = tol, maxiter
        self.glt = None
        if post_smoother == "glt":
            from .splines import array_to_mat_stencil, collocation_cardinal_splines
            Cm = array_to_mat_stencil(n, p, collocation_cardinal_splines(p, n))
            self.glt = [Cm] * ndim

    @property
    def ndof(self) -> int:
        return self.space.dimension

    def rhs_ones(self) -> StencilVector:
        """``bf[i] = 1`` on every owned coefficient (`sources/mg_jac.py:57-62`)."""
        b = self.space.empty()
        _lib.call("poms_vec_fill", self.space.ctx, C.byref(self.space.layout), 1.0, rt.ptr(b._data),
                  rt.stream_handle())
        b._mark_written()
        b.update_ghost_regions()
        return b

    def coarse_solve(self, rc: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        _lib.call("poms_dense_matvec", self.space.ctx, rc.numel(), rt.ptr(self.Ainv), rt.ptr(rc),
                  rt.ptr(out), rt.stream_handle())
        return out

    def cycle(self, bf: StencilVector, x0: StencilVector | None = None):
        """One V-cycle; returns ``(xf2, info_pre, info_pos)``."""
        A = self.A
        xf, info_pre = pcg(A, damped_jacobi, bf, x0=x0, tol=self.tol, maxiter=self.maxiter)
        if self.fused_restrict:
            rc = self.transfer.resid_restrict(A, bf, xf, out=self.rc)
        else:
            rf = A.residual(bf, xf)
            rc = self.transfer.restrict(rf, out=self.rc)
        xc = self.coarse_solve(rc, self.xc)
        self.transfer.prolong_add(xc, xf)
        xf.update_ghost_regions()
        if self.glt is not None:
            from .solvers import pcg_kron
            xf2, info_pos = pcg_kron(A, self.glt, bf, x0=xf, tol=self.tol, maxiter=self.p + 1)
        else:
            # (xf is this cycle's own temporary: iterate in its buffer, no copy)
            xf2, info_pos = pcg(A, damped_jacobi, bf, x0=xf, tol=self.tol, maxiter=self.maxiter, _x0_owned=True)
        return xf2, info_pre, info_pos


class MultilevelVCycle:
    """V-cycle over a hierarchy of nested uniform B-spline spaces (SURVEY §8f
    rank 1: the reference's two-level cycle `sources/mg_jac.py:84-119` applied
    recursively, with every level's operator, smoothing and transfers on the
    device and a dense device solve on the coarsest level).

    Level 0 has ``ncells_fine`` cells per axis; each coarser level halves the
    cells (dyadic knot insertion, ``P1 = matrix_multi_stages``) down to
    ``ncells_coarsest``.  Level operators are assembled on their own knots; for
    nested spaces with exact quadrature that IS the Galerkin product R A P of
    the reference (pinned by tests/test_splines.py and the oracle parity test).
    Each level is smoothed by ``pcg(A_l, damped_jacobi, b_l, tol, maxiters[l])``
    before and after the coarse correction, as the reference smooths its fine
    level.  With ``dist`` the finest level is slab-decomposed; the restriction
    to level 1 is all-reduced and the coarser levels are replicated on every
    rank (their work is 1/8, 1/64, ... of the finest level's).
    """

    def __init__(self, p: int, ncells_fine: int, ncells_coarsest: int = 8, ndim: int = 3, *,
                 dist=None, mass_coef: float = 1.0, device=None, tol: float = 1e-6, maxiters=None,
                 align: bool = True, chunk: int = 0, fused_restrict: bool | None = None):
        if ncells_fine < ncells_coarsest or ncells_coarsest < 1:
            raise ValueError("need ncells_fine >= ncells_coarsest >= 1")
        self.p, self.ndim, self.tol = int(p), int(ndim), tol
        cells = [int(ncells_fine)]
        while cells[-1] // 2 >= ncells_coarsest and cells[-1] % 2 == 0:
            cells.append(cells[-1] // 2)
        if len(cells) < 2:
            raise ValueError("the hierarchy needs at least two levels (even cell counts)")
        self.cells = cells
        self.nlevels = L = len(cells)
        self.maxiters = [10] * (L - 1) if maxiters is None else [int(m) for m in maxiters]
        if len(self.maxiters) != L - 1:
            raise ValueError(f"maxiters needs {L - 1} entries")
        knots = [uniform_knots(p, N) for N in cells]
        self.knots = knots
        self.P1 = []
        self.M1d, self.K1d, self.spaces, self.ops, self.transfers = [], [], [], [], []
        for l in range(L):
            n = len(knots[l]) - p - 1
            M, K = assemble_1d(knots[l], p)
            self.M1d.append(M)
            self.K1d.append(K)
            if l < L - 1:
                _, _, P1 = two_level_setup_1d(p, knots[l], knots[l + 1])
                self.P1.append(P1)
            if l == L - 1:
                break
            V = StencilVectorSpace([n] * ndim, [p] * ndim, dist=dist if l == 0 else None, device=device,
                                   align=align)
            A = KronOperator.laplace(V, [M] * ndim, [K] * ndim, mass_coef=mass_coef)
            if chunk:
                A.set_chunk(chunk)
            self.spaces.append(V)
            self.ops.append(A)
            self.transfers.append(KronTransfer(V, [self.P1[l]] * ndim))
        # fused residual -> restriction where the transfer is dense (coarse extents <= 32);
        # None: in 3D (as TwoLevelVCycle)
        if fused_restrict is None:
            fused_restrict = ndim == 3
        self.fused = [bool(fused_restrict) and tr.set_operator(A) for tr, A in zip(self.transfers, self.ops)]
        # coarsest level: dense inverse of its operator (assembled = Galerkin, nested)
        from .splines import band_to_dense
        Mc, Kc = band_to_dense(self.M1d[-1]), band_to_dense(self.K1d[-1])
        Ac = galerkin_coarse_dense(Mc, Kc, ndim, mass_coef)
        self.Ac = Ac
        Ainv = sla.lu_solve(sla.lu_factor(Ac), np.eye(Ac.shape[0]))
        dev = f"cuda:{self.spaces[0].device}"
        self.Ainv = torch.from_numpy(np.ascontiguousarray(Ainv)).to(dev)
        self.rcs = [torch.empty(tr.ncoarse, dtype=F64, device=dev) for tr in self.transfers]
        self.xc = torch.empty(Ac.shape[0], dtype=F64, device=dev)
        self.infos = [None] * (L - 1)

    @property
    def ndof(self) -> int:
        return self.spaces[0].dimension

    @property
    def space(self) -> StencilVectorSpace:
        return self.spaces[0]

    @property
    def A(self) -> KronOperator:
        return self.ops[0]

    def rhs_ones(self) -> StencilVector:
        b = self.spaces[0].empty()
        _lib.call("poms_vec_fill", self.spaces[0].ctx, C.byref(self.spaces[0].layout), 1.0, rt.ptr(b._data),
                  rt.stream_handle())
        b._mark_written()
        b.update_ghost_regions()
        return b

    def _level(self, l: int, b: StencilVector, x0: StencilVector | None) -> StencilVector:
        A, tr = self.ops[l], self.transfers[l]
        x, ipre = pcg(A, damped_jacobi, b, x0=x0, tol=self.tol, maxiter=self.maxiters[l])
        if self.fused[l]:
            rc = tr.resid_restrict(A, b, x, out=self.rcs[l])
        else:
            rc = tr.restrict(A.residual(b, x), out=self.rcs[l])
        if l + 1 == self.nlevels - 1:
            ec = self.xc
            _lib.call("poms_dense_matvec", self.spaces[0].ctx, rc.numel(), rt.ptr(self.Ainv), rt.ptr(rc),
                      rt.ptr(ec), rt.stream_handle())
        else:
            Vc = self.spaces[l + 1]
            bc = Vc.empty()
            Vc.interior(bc._data).copy_(rc.view(Vc.local_npts))
            bc._mark_written()
            bc.update_ghost_regions()
            ecv = self._level(l + 1, bc, None)
            ec = Vc.interior(ecv._data).contiguous().view(-1)
        tr.prolong_add(ec, x)
        x.update_ghost_regions()
        x, ipos = pcg(A, damped_jacobi, b, x0=x, tol=self.tol, maxiter=self.maxiters[l])
        if self.infos[l] is None:
            self.infos[l] = (ipre, ipos)
        return x

    def cycle(self, b: StencilVector, x0: StencilVector | None = None):
        """One V-cycle from level 0; returns ``(x, infos)``, ``infos[l] = (info_pre,
        info_post)`` of level l's first visit in this cycle."""
        self.infos = [None] * (self.nlevels - 1)
        x = self._level(0, b, x0)
        return x, list(self.infos)

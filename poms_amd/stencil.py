"""Device-backed, spl-compatible stencil types.

The reference solvers (`sources/solvers.py`) duck-type spl's
``StencilVectorSpace`` / ``StencilVector`` / ``StencilMatrix``
(SURVEY §8b): ``A.shape``, ``A.dot(x)``, ``A[i1, i2, 0, 0]``;
``v.space.starts/ends/pads/npts``, ``v[:, :] = c``, ``v[i1, i2]``,
``v.copy()``, ``a*v``, ``v + w``, ``v - w``, ``v.dot(w)``,
``v.update_ghost_regions()``, ``v.toarray()``.  These classes provide that
surface over HBM-resident padded arrays (the spl ``_data`` layout,
`slides/content.tex:256-264`), and dispatch whole-vector work to
``libpoms_hip.so``.  Per-element ``__getitem__``/``__setitem__`` exist for API
parity only (each is a device round trip).

``KronOperator`` is the banded Kronecker(-sum) operator: the V-cycle's fine
matrix (the assembled ``-Δu + u`` of `sources/matrix_assembler.py:84-179`,
applied by spl ``StencilMatrix.dot``) and the ``(A, B)`` pair of
``kron_dot_v2`` (`sources/kron_product.py:56-89`).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Sequence

import numpy as np
import torch

from . import _lib
from . import runtime as rt
from .dist import CartDistribution, SlabDistribution

F64 = torch.float64


class StencilVectorSpace:
    """Padded, possibly slab-distributed, 1D/2D/3D vector space on one GPU.

    ``npts``: global number of coefficients per axis; ``pads``: ghost width per
    axis (the spline degree).  Non-periodic only -- every driver of the
    reference is non-periodic (`sources/mg_jac.py`).  With
    ``dist`` a :class:`SlabDistribution` splits the slowest axis into slabs (3D
    only); a :class:`CartDistribution` splits every axis into blocks (spl ``Cart``).
    """

    def __init__(self, npts: Sequence[int], pads: Sequence[int], periods=None, *,
                 dist: SlabDistribution | CartDistribution | None = None, device=None, align: bool = False):
        npts, pads = tuple(int(v) for v in npts), tuple(int(v) for v in pads)
        if not 1 <= len(npts) <= 3 or len(pads) != len(npts):
            raise ValueError("npts/pads must have 1..3 equal-length entries")
        if periods is not None and any(periods):
            raise NotImplementedError("periodic spaces are not supported (reference drivers are non-periodic)")
        if any(n < 1 for n in npts) or any(p < 0 for p in pads):
            raise ValueError("bad npts/pads")
        self.is_cart = isinstance(dist, CartDistribution)
        if self.is_cart:
            if dist.npts != npts:
                raise ValueError(f"distribution npts {dist.npts} do not match {npts}")
            for d, (nl, p, g) in enumerate(zip(dist.n_local, pads, dist.dims)):
                if g > 1 and nl < p:
                    raise ValueError(f"axis {d}: block of {nl} points is thinner than the pad {p}")
        elif dist is not None:
            if len(npts) != 3:
                raise NotImplementedError("slab distribution is implemented for 3D spaces")
            if dist.n0_global != npts[0]:
                raise ValueError("distribution does not match npts[0]")
        self.npts, self.pads, self.ndim = npts, pads, len(npts)
        self.periods = (False,) * self.ndim
        self.dist = dist
        if self.is_cart:
            self.starts = tuple(dist.starts)
            self.ends = tuple(e - 1 for e in dist.ends)
        else:
            s0, e0 = (dist.start, dist.end - 1) if dist is not None else (0, npts[0] - 1)
            self.starts = (s0,) + (0,) * (self.ndim - 1)
            self.ends = (e0,) + tuple(n - 1 for n in npts[1:])
        self.local_npts = tuple(e - s + 1 for s, e in zip(self.starts, self.ends))
        lead = 3 - self.ndim
        self.n3 = (1,) * lead + self.local_npts
        self.p3 = (0,) * lead + self.pads
        self.padded_shape = tuple(n + 2 * p for n, p in zip(self.local_npts, self.pads))
        # HBM layout.  With ``align`` rows of axis 2 are `pitch` doubles apart (a
        # multiple of 16 = one 128-B line) and the array starts `shift` doubles into
        # its buffer, so interior column 0 of every row starts a line and a tile
        # whose output columns are a multiple of 16 stores whole lines only.  Off by
        # default: measured no faster at 515^3 (profiles/r01/align/), while the
        # 48-column tiles it needs cost 10-15 % (more halo lanes).
        n2p = self.padded_shape[-1]
        self.aligned = bool(align) and self.ndim >= 2
        if self.aligned:
            self.pitch = -(-n2p // 16) * 16
            self.shift = (16 - self.pads[-1] % 16) % 16
        else:
            self.pitch, self.shift = n2p, 0
        lead_shape = self.padded_shape[:-1]
        self.strides = tuple(int(np.prod(lead_shape[i + 1:])) * self.pitch for i in range(len(lead_shape))) + (1,)
        self.plane_elems = self.strides[0] if self.ndim == 3 else int(np.prod(lead_shape)) * self.pitch
        self.store_elems = self.padded_shape[0] * self.strides[0] + self.shift + (16 if self.aligned else 0)
        # a Cart block's ghost rows / columns (axes 1, 2) hold the neighbours' data
        ghost_data = self.is_cart and any(g > 1 for g in dist.dims[-2:])
        self.layout = _lib.Layout.make(self.n3, self.p3, self.pitch if self.aligned else 0,
                                       _lib.LAYOUT_GHOST_DATA if ghost_data else 0)
        self.dimension = int(np.prod(npts))
        self.device = rt.device_index(device)
        self.ctx = rt.ctx(self.device)
        self._scal = None
        self._pinned = None

    # ------------------------------------------------------------------
    @property
    def is_distributed(self) -> bool:
        return self.dist is not None and self.dist.world > 1

    def interior(self, data: torch.Tensor) -> torch.Tensor:
        """View of the owned (interior) entries of a padded array."""
        return data[tuple(slice(p, p + n) for p, n in zip(self.pads, self.local_npts))]

    def zeros(self) -> "StencilVector":
        return StencilVector(self)

    def view(self, store: torch.Tensor) -> torch.Tensor:
        """The padded array (``padded_shape``) inside a flat buffer of ``store_elems``."""
        return torch.as_strided(store, self.padded_shape, self.strides, self.shift)

    def planes(self, store: torch.Tensor) -> torch.Tensor:
        """The padded array as contiguous rows of whole axis-0 planes (3D), for the
        slab ghost exchange (a plane includes its dead row-pitch columns)."""
        return torch.as_strided(store, (self.padded_shape[0], self.plane_elems), (self.plane_elems, 1), self.shift)

    def empty(self) -> "StencilVector":
        """Vector with unspecified interior and zero ghost cells (no full memset)."""
        store = torch.empty(self.store_elems, dtype=F64, device=f"cuda:{self.device}")
        # ghost planes / rows / columns and dead pitch columns (finite, never NaN) in one launch
        _lib.call("poms_vec_zero_ghosts", self.ctx, C.byref(self.layout), rt.ptr(self.view(store)),
                  rt.stream_handle())
        return StencilVector(self, _store=store)

    def scalar_buffer(self) -> torch.Tensor:
        if self._scal is None:
            self._scal = torch.zeros(8, dtype=F64, device=f"cuda:{self.device}")
        return self._scal

    @property
    def lazy_reductions(self) -> bool:
        """Global sums can stay on the device stream (single rank, or RCCL)."""
        return not self.is_distributed or bool(self.dist.device_reductions)

    def _side_stream(self) -> torch.cuda.Stream:
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=f"cuda:{self.device}")
        return self._side

    def lazy_sum(self, *partial_sums: torch.Tensor) -> "LazyScalar":
        """Global sums of device partial-sum slices, copied to pinned host memory
        without blocking the host; ``.value(i)`` waits for that copy only.

        The local sums are snapshotted on the launch stream (the partial-sum
        buffer is reused by the next launch); the RCCL all-reduce and the copy run
        on a side stream, so the next sweep never waits for them."""
        if not self.is_distributed and len(partial_sums) == 1:
            # one rank, already reduced on the device: one async copy to pinned memory
            # (no torch ops: this runs ~220 times per V-cycle)
            src = partial_sums[0]
            return self._lazy_copy_raw(src)
        tot = torch.stack([ps.sum() for ps in partial_sums]) if len(partial_sums) > 1 else partial_sums[0].clone()
        if self.is_distributed and self.dist.native is not None:
            # native RCCL: all-reduce and the copy to pinned memory both on the
            # communication stream; the launch stream never waits for them
            nc = self.dist.native
            nc.allreduce(tot, rt.stream_handle(), wait_back=False)
            tot.record_stream(nc.stream)
            with torch.cuda.stream(nc.stream):
                return self._lazy_copy(tot)
        side = self._side_stream()
        side.wait_stream(torch.cuda.current_stream(tot.device))
        tot.record_stream(side)
        with torch.cuda.stream(side):
            if self.is_distributed:
                import torch.distributed as dist
                dist.all_reduce(tot, group=self.dist.group)
            return self._lazy_copy(tot)

    def pinned_slots(self, k: int) -> torch.Tensor:
        """k doubles of the pinned host ring (each use is read within a few sweeps)."""
        if self._pinned is None:
            self._pinned = torch.zeros(8, dtype=F64).pin_memory()
            self._pin_next = 0
        if self._pin_next + k > 8:
            self._pin_next = 0
        slot = self._pinned[self._pin_next:self._pin_next + k]
        self._pin_next += k
        return slot

    def _lazy_copy_raw(self, src: torch.Tensor) -> "LazyScalar":
        """hipMemcpyAsync of a (contiguous) device slice into the pinned ring, on the
        launch stream, and an event after it."""
        if self._pinned is None:
            self._pinned = torch.zeros(8, dtype=F64).pin_memory()
            self._pin_next = 0
        k = src.numel()
        if self._pin_next + k > 8:
            self._pin_next = 0
        slot = self._pinned[self._pin_next:self._pin_next + k]
        self._pin_next += k
        _lib.call("poms_copy_to_host_async", self.ctx, rt.ptr(src), rt.ptr(slot), k, rt.stream_handle())
        return LazyScalar(None, slot)

    def _lazy_copy(self, tot: torch.Tensor) -> "LazyScalar":
        if self._pinned is None:
            self._pinned = torch.zeros(8, dtype=F64).pin_memory()
            self._pin_next = 0
        k = tot.numel()
        if self._pin_next + k > 8:
            self._pin_next = 0
        slot = self._pinned[self._pin_next:self._pin_next + k]
        self._pin_next += k
        return LazyScalar(tot, slot)

    def device_sum(self, *partial_sums: torch.Tensor) -> torch.Tensor:
        """Global sums of device partial-sum slices as a device tensor (RCCL all-reduce
        across slabs on the device stream; nothing is read by the host)."""
        tot = torch.stack([ps.sum() for ps in partial_sums]) if len(partial_sums) > 1 else partial_sums[0].clone()
        if self.is_distributed:
            if self.dist.native is not None:
                self.dist.native.allreduce(tot, rt.stream_handle(), wait_back=True)
            else:
                import torch.distributed as dist
                dist.all_reduce(tot, group=self.dist.group)
        return tot

    def lazy_value(self, dev: torch.Tensor) -> "LazyScalar":
        """Copy a device scalar tensor to pinned host memory without blocking.

        Its own ring (apart from :meth:`lazy_sum`'s), so that the damped-Jacobi
        norms queued after it cannot overwrite the slot before it is read."""
        if getattr(self, "_pinned_v", None) is None:
            self._pinned_v = torch.zeros(8, dtype=F64).pin_memory()
            self._pinv_next = 0
        k = dev.numel()
        if self._pinv_next + k > 8:
            self._pinv_next = 0
        slot = self._pinned_v[self._pinv_next:self._pinv_next + k]
        self._pinv_next += k
        return LazyScalar(dev, slot)

    def global_dot(self, local: float) -> float:
        if self.is_distributed:
            comm = rt.Comm.from_env(self.dist.group)
            return comm.allreduce_scalar(local)
        return local

    def __repr__(self):
        return f"StencilVectorSpace(npts={self.npts}, pads={self.pads}, starts={self.starts}, ends={self.ends})"


class LazyScalar:
    """A device scalar being copied to pinned host memory on the launch stream."""

    def __init__(self, dev_value: torch.Tensor | None, host_slot: torch.Tensor):
        if dev_value is not None:   # else the caller already queued the copy
            host_slot.copy_(dev_value, non_blocking=True)
        self._ev = torch.cuda.Event()
        self._ev.record()
        self._host = host_slot

    def value(self, i: int = 0) -> float:
        self._ev.synchronize()
        return float(self._host[i])


def _stream():
    return rt.stream_handle()


class StencilVector:
    """Vector of a :class:`StencilVectorSpace`, stored padded in HBM."""

    __array_priority__ = 100

    def __init__(self, V: StencilVectorSpace, *, _store: torch.Tensor | None = None):
        self._space = V
        if _store is None:
            _store = torch.zeros(V.store_elems, dtype=F64, device=f"cuda:{V.device}")
        if _store.dim() != 1 or _store.numel() != V.store_elems or _store.dtype != F64 or not _store.is_contiguous():
            raise ValueError("buffer does not match the space layout")
        self._store = _store
        self._data = V.view(_store)
        self._ghost_valid = True

    # -- spl surface ----------------------------------------------------
    @property
    def space(self) -> StencilVectorSpace:
        return self._space

    @property
    def shape(self):
        return (self._space.dimension,)

    @property
    def starts(self):
        return self._space.starts

    @property
    def ends(self):
        return self._space.ends

    @property
    def pads(self):
        return self._space.pads

    def _mark_written(self):
        self._ghost_valid = not self._space.is_distributed

    def copy(self) -> "StencilVector":
        out = StencilVector(self._space, _store=self._store.clone())
        out._ghost_valid = self._ghost_valid
        return out

    def assign(self, other: "StencilVector") -> "StencilVector":
        """self <- other (interior), no allocation."""
        _lib.call("poms_vec_scale", self._space.ctx, C.byref(self._space.layout), 1.0,
                  rt.ptr(other._data), rt.ptr(self._data), _stream())
        self._mark_written()
        return self

    def axpby_(self, a: float, x: "StencilVector", b: float) -> "StencilVector":
        """self <- a*x + b*self (interior)."""
        _lib.call("poms_vec_axpby", self._space.ctx, C.byref(self._space.layout), float(a),
                  rt.ptr(x._data), float(b), rt.ptr(self._data), rt.ptr(self._data), _stream())
        self._mark_written()
        return self

    def _lin(self, a: float, other, b: float) -> "StencilVector":
        out = self._space.empty()
        if other is None:
            _lib.call("poms_vec_scale", self._space.ctx, C.byref(self._space.layout), float(a),
                      rt.ptr(self._data), rt.ptr(out._data), _stream())
        else:
            if not isinstance(other, StencilVector) or other._space is not self._space:
                raise TypeError("operands must belong to the same StencilVectorSpace")
            _lib.call("poms_vec_axpby", self._space.ctx, C.byref(self._space.layout), float(a),
                      rt.ptr(self._data), float(b), rt.ptr(other._data), rt.ptr(out._data), _stream())
        out._mark_written()
        return out

    def __add__(self, other):
        return self._lin(1.0, other, 1.0)

    def __sub__(self, other):
        return self._lin(1.0, other, -1.0)

    def __mul__(self, a):
        if not isinstance(a, (int, float, np.floating, np.integer)):
            return NotImplemented
        return self._lin(float(a), None, 0.0)

    __rmul__ = __mul__

    def __neg__(self):
        return self._lin(-1.0, None, 0.0)

    def __iadd__(self, other):
        _lib.call("poms_vec_axpby", self._space.ctx, C.byref(self._space.layout), 1.0,
                  rt.ptr(self._data), 1.0, rt.ptr(other._data), rt.ptr(self._data), _stream())
        self._mark_written()
        return self

    def __isub__(self, other):
        _lib.call("poms_vec_axpby", self._space.ctx, C.byref(self._space.layout), 1.0,
                  rt.ptr(self._data), -1.0, rt.ptr(other._data), rt.ptr(self._data), _stream())
        self._mark_written()
        return self

    def __imul__(self, a):
        _lib.call("poms_vec_scale", self._space.ctx, C.byref(self._space.layout), float(a),
                  rt.ptr(self._data), rt.ptr(self._data), _stream())
        self._mark_written()
        return self

    def dot_device(self, other: "StencilVector") -> torch.Tensor:
        """Global inner product as a device tensor of shape (1,) (no host read)."""
        V = self._space
        buf = V.scalar_buffer()
        _lib.call("poms_vec_dot", V.ctx, C.byref(V.layout), rt.ptr(self._data), rt.ptr(other._data),
                  rt.ptr(buf), _stream())
        return V.device_sum(buf[0:1])

    def dot(self, other: "StencilVector") -> float:
        """Global inner product (RCCL all-reduce across slabs), as spl ``StencilVector.dot``."""
        V = self._space
        buf = V.scalar_buffer()
        _lib.call("poms_vec_dot", V.ctx, C.byref(V.layout), rt.ptr(self._data), rt.ptr(other._data),
                  rt.ptr(buf), _stream())
        return V.global_dot(float(buf[0].item()))

    def update_ghost_regions(self, direction=None) -> None:
        V = self._space
        if V.is_distributed and V.is_cart:
            if direction is None:
                V.dist.exchange(self._data, V.pads)
                self._ghost_valid = True
            else:   # one axis only (spl's per-direction update)
                V.dist.exchange(self._data, V.pads, [V.pads[d] if d == direction else 0 for d in range(V.ndim)])
            return
        if V.is_distributed and (direction is None or direction == 0):
            V.dist.exchange(V.planes(self._store), width=V.pads[0], pad=V.pads[0])
            self._ghost_valid = True

    def toarray(self) -> np.ndarray:
        """Global-size flat array holding this rank's entries (zeros elsewhere)."""
        V = self._space
        out = np.zeros(V.npts)
        loc = V.interior(self._data).cpu().numpy()
        out[tuple(slice(s, e + 1) for s, e in zip(V.starts, V.ends))] = loc
        return out.reshape(-1)

    def to_local_numpy(self) -> np.ndarray:
        return self._space.interior(self._data).cpu().numpy()

    def from_numpy(self, arr: np.ndarray) -> "StencilVector":
        """Set the owned entries from a global-shaped (or local-shaped) array."""
        V = self._space
        arr = np.asarray(arr, dtype=np.float64)
        if arr.shape == V.npts:
            arr = arr[tuple(slice(s, e + 1) for s, e in zip(V.starts, V.ends))]
        if arr.shape != V.local_npts:
            raise ValueError(f"array shape {arr.shape} matches neither {V.npts} nor {V.local_npts}")
        V.interior(self._data).copy_(torch.from_numpy(np.ascontiguousarray(arr)))
        self._mark_written()
        return self

    # -- element access with spl's global indices -------------------------------
    def _index(self, key):
        V = self._space
        if not isinstance(key, tuple):
            key = (key,)
        if len(key) != V.ndim:
            raise IndexError("need one index per axis")
        out = []
        for k, s, e, p in zip(key, V.starts, V.ends, V.pads):
            if isinstance(k, slice):
                if k == slice(None):
                    out.append(slice(p, p + e - s + 1))
                else:
                    a = s if k.start is None else k.start
                    b = e + 1 if k.stop is None else k.stop
                    out.append(slice(a - s + p, b - s + p, k.step))
            else:
                out.append(int(k) - s + p)
        return tuple(out)

    def __getitem__(self, key):
        v = self._data[self._index(key)]
        return float(v.item()) if v.dim() == 0 else v.cpu().numpy()

    def __setitem__(self, key, value):
        self._data[self._index(key)] = torch.as_tensor(value, dtype=F64)
        self._mark_written()

    def __repr__(self):
        return f"StencilVector({self._space!r})"


class StencilMatrix1D:
    """Host 1D banded ``StencilMatrix`` (spl layout ``M[i, k]``, ``k in [-p, p]``).

    Used to hand band factors to :func:`poms_amd.kron_product.kron_dot_v2`
    (as `sources/tests/test_kron_dot.py:21-29` builds them).
    """

    def __init__(self, n: int, p: int, band: np.ndarray | None = None):
        self.n, self.p = int(n), int(p)
        self.band = np.zeros((self.n, 2 * self.p + 1)) if band is None else np.array(band, dtype=np.float64)
        if self.band.shape != (self.n, 2 * self.p + 1):
            raise ValueError("band shape mismatch")

    starts = property(lambda self: (0,))
    ends = property(lambda self: (self.n - 1,))
    pads = property(lambda self: (self.p,))
    shape = property(lambda self: (self.n, self.n))

    def __getitem__(self, key):
        i, k = key
        return self.band[i, k + self.p]

    def __setitem__(self, key, value):
        i, k = key
        if isinstance(i, slice):
            self.band[i, k + self.p] = value
        else:
            self.band[i, k + self.p] = value

    def remove_spurious_entries(self):
        for i in range(self.n):
            for k in range(-self.p, self.p + 1):
                if not 0 <= i + k < self.n:
                    self.band[i, k + self.p] = 0.0

    def toarray(self) -> np.ndarray:
        from .splines import band_to_dense
        return band_to_dense(self.band)

    def tocsr(self):
        import scipy.sparse as sp
        return sp.csr_matrix(self.toarray())


def _band_of(F) -> np.ndarray:
    if isinstance(F, StencilMatrix1D):
        return F.band
    b = np.asarray(F, dtype=np.float64)
    if b.ndim != 2 or b.shape[1] % 2 != 1:
        raise ValueError("band factor must be (n, 2p+1)")
    return b


def _widen(band: np.ndarray, pmax: int) -> np.ndarray:
    n, w = band.shape
    p = (w - 1) // 2
    out = np.zeros((n, 2 * pmax + 1))
    out[:, pmax - p:pmax + p + 1] = band
    return np.ascontiguousarray(out)


def _unit_band(pmax: int, value: float = 1.0) -> np.ndarray:
    b = np.zeros((1, 2 * pmax + 1))
    b[0, pmax] = value
    return b


class KronOperator:
    """Banded Kronecker(-sum) operator on a :class:`StencilVectorSpace`.

    ``form='sum'``:  A = c M⊗M⊗M + K⊗M⊗M + M⊗K⊗M + M⊗M⊗K  (``-Δu + c u`` with
    natural BCs; 2D/1D analogues).  ``form='single'``: A = F0⊗F1⊗F2.
    """

    def __init__(self, V: StencilVectorSpace, form: str, bands: dict, pmax: int):
        self.space, self.form = V, form
        self.pmax = int(pmax)
        self.bands = bands  # host copies (global rows) by role name
        self._h = C.c_void_p()
        nd = V.ndim
        W = 2 * self.pmax + 1
        keep = []

        def arr(b):
            a = np.ascontiguousarray(b, dtype=np.float64)
            assert a.shape[1] == W
            keep.append(a)
            return a.ctypes.data_as(C.c_void_p)

        # factor rows of this rank: axis 0 of a 3D space is passed whole (the device
        # tables are indexed by global plane, g0); with a Cart block the rows of the
        # other axes are sliced to the owned block (its neighbours' rows act through
        # the exchanged ghosts)
        role_axis = {"A1": nd - 2, "B1": nd - 2, "F1": nd - 2, "M2": nd - 1, "K2": nd - 1, "F2": nd - 1}

        def rows(name):
            b = bands[name]
            ax = role_axis.get(name, -1)
            if not V.is_cart or ax < 0 or b.shape[0] == 1:
                return b
            return b[V.starts[ax]:V.ends[ax] + 1]

        f = [None] * 6
        if form == "sum":
            if nd == 3:
                f[0], f[1] = arr(bands["A0"]), arr(bands["M0"])
            f[2], f[3], f[4], f[5] = arr(rows("A1")), arr(rows("B1")), arr(rows("M2")), arr(rows("K2"))
            cform = _lib.FORM_SUM
        else:
            if nd == 3:
                f[0] = arr(bands["F0"])
            f[2], f[4] = arr(rows("F1")), arr(rows("F2"))
            cform = _lib.FORM_SINGLE
        farr = (C.c_void_p * 6)(*f)
        g0 = V.starts[0] if nd == 3 else 0
        n0g = V.npts[0] if nd == 3 else 1
        _lib.call("poms_op_create", V.ctx, 3 if nd == 3 else 2, C.byref(V.layout), cform, self.pmax,
                  farr, g0, n0g, C.byref(self._h))
        d = V.dist if V.is_distributed else None
        if d is not None and getattr(d, "native", None) is not None and d.native.peer and nd == 3:
            # peer transport: the mailboxes for this operator's exchanges now, on every
            # rank (operators are built in the same order everywhere), not inside a capture
            d.native.peer_reserve(self.pmax * V.plane_elems, -1 if d.prev is None else d.prev,
                                  -1 if d.next is None else d.next)
        self.timer = None  # list -> (kind, start_event, end_event, call) per kernel launch
        self._calls = 0    # operator calls (one call = 1 launch, or 2 when a halo exchange is overlapped)

    # -- constructors ------------------------------------------------------------
    @classmethod
    def laplace(cls, V: StencilVectorSpace, M: Sequence, K: Sequence, mass_coef: float = 1.0):
        """-Δu + c u in Kronecker-sum form from per-axis 1D (mass, stiffness) bands."""
        nd = V.ndim
        M = [_band_of(m) for m in M]
        K = [_band_of(k) for k in K]
        if len(M) != nd or len(K) != nd:
            raise ValueError("need one (M, K) pair per axis")
        for d in range(nd):
            if M[d].shape[0] != V.npts[d] or K[d].shape != M[d].shape:
                raise ValueError(f"axis {d}: factor rows do not match npts")
        pmax = max(max((m.shape[1] - 1) // 2 for m in M), max(V.pads), 1)
        Mw = [_widen(m, pmax) for m in M]
        Kw = [_widen(k, pmax) for k in K]
        c = float(mass_coef)
        if nd == 3:
            bands = {"A0": c * Mw[0] + Kw[0], "M0": Mw[0], "A1": Mw[1], "B1": Kw[1], "M2": Mw[2], "K2": Kw[2]}
        elif nd == 2:
            bands = {"A1": c * Mw[0] + Kw[0], "B1": Mw[0], "M2": Mw[1], "K2": Kw[1]}
        else:
            bands = {"A1": _unit_band(pmax, c), "B1": _unit_band(pmax, 1.0), "M2": Mw[0], "K2": Kw[0]}
        op = cls(V, "sum", bands, pmax)
        op.M, op.K, op.mass_coef = M, K, c
        return op

    @classmethod
    def product(cls, V: StencilVectorSpace, F: Sequence):
        """Single Kronecker product F0⊗F1(⊗F2) (``kron_dot``)."""
        nd = V.ndim
        F = [_band_of(f) for f in F]
        if len(F) != nd:
            raise ValueError("need one factor per axis")
        for d in range(nd):
            if F[d].shape[0] != V.npts[d]:
                raise ValueError(f"axis {d}: factor rows do not match npts")
        pmax = max(max((f.shape[1] - 1) // 2 for f in F), max(V.pads), 1)
        Fw = [_widen(f, pmax) for f in F]
        if nd == 3:
            bands = {"F0": Fw[0], "F1": Fw[1], "F2": Fw[2]}
        elif nd == 2:
            bands = {"F1": Fw[0], "F2": Fw[1]}
        else:
            bands = {"F1": _unit_band(pmax), "F2": Fw[0]}
        op = cls(V, "single", bands, pmax)
        op.F = F
        return op

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib.poms_op_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- spl surface -------------------------------------------------------------
    @property
    def shape(self):
        return (self.space.dimension, self.space.dimension)

    def set_chunk(self, chunk: int) -> None:
        _lib.call("poms_op_set_chunk", self._h, int(chunk))

    def set_tile_cols(self, cols: int) -> None:
        """Output columns per 64-lane tile of the v3/v4 kernels (0 = 64 - 2 pmax)."""
        _lib.call("poms_op_set_tile_cols", self._h, int(cols))

    def set_variant(self, variant: int) -> None:
        """0 general, 4/9 v3, 7 v4, 10 v5, 8 auto (see poms_hip.h)."""
        _lib.call("poms_op_set_variant", self._h, int(variant))

    @property
    def variant(self) -> int:
        v = C.c_int()
        _lib.call("poms_op_get_variant", self._h, C.byref(v))
        return v.value

    EPILOGUES = {"apply": 0, "residual": 1, "jacobi": 2, "jacobi_from_zero": 3, "apply_dot": 4}

    def timing(self, enable: bool = True, epilogue: str | None = None, every: int = 1, reserve: int = 0) -> None:
        """Bracket launches of this operator (any caller, the native pcg loop included)
        with HIP events on their stream: those of ``epilogue`` (None: all), every
        ``every``-th; enabling clears the record and pre-creates ``reserve`` event pairs."""
        _lib.call("poms_op_timing", self._h, 1 if enable else 0, -1 if epilogue is None else self.EPILOGUES[epilogue],
                  int(every), int(reserve))

    def timing_read(self, epilogue: str):
        """(seconds, launches, output DOFs) of the recorded launches of one epilogue."""
        ms, n, d = C.c_double(), C.c_int64(), C.c_int64()
        _lib.call("poms_op_timing_read", self._h, self.EPILOGUES[epilogue], C.byref(ms), C.byref(n), C.byref(d))
        return ms.value * 1e-3, n.value, d.value

    @property
    def last_variant(self) -> int:
        """Variant the last launch ran (after the per-call fall-backs; -1 before any)."""
        v = C.c_int()
        _lib.call("poms_op_last_variant", self._h, C.byref(v))
        return v.value

    @property
    def spec_stats(self) -> dict:
        """The native smoother's speculative calls: calls, repeats (a stop test fired,
        the call ran again step by step), graph captures and graph replays."""
        v = (C.c_int * 4)()
        _lib.call("poms_op_spec_stats", self._h, v)
        return {"calls": v[0], "repeats": v[1], "captures": v[2], "replays": v[3]}

    def kernel_variant(self, epilogue: str) -> int:
        """Variant one launch of ``epilogue`` runs after auto-selection / fall-backs."""
        v = C.c_int()
        _lib.call("poms_op_kernel_variant", self._h, self.EPILOGUES[epilogue], C.byref(v))
        return v.value

    def _check(self, *vs):
        for v in vs:
            if not isinstance(v, StencilVector) or v.space is not self.space:
                raise TypeError("vector does not belong to this operator's space")

    # epilogue codes of poms_op_run_reduce
    _EPI = {"apply": 0, "residual": 1, "jacobi": 2, "jacobi2": 3, "apply_dot": 4, "sweep2": 6}

    def _run(self, kind: str, x: StencilVector, y: StencilVector, b: StencilVector | None = None,
             omega: float = 0.0, norm_out: torch.Tensor | None = None, dot_out: torch.Tensor | None = None):
        """One operator call over all local planes (``poms_op_run_reduce2``); with
        stale ghosts in a slab decomposition the RCCL ghost exchange overlaps the
        interior planes, and the p boundary planes on both sides follow in one launch.  The
        reductions of the launches accumulate into ``norm_out`` / ``dot_out``
        (device doubles)."""
        V = self.space
        if V.is_distributed and V.dist.native is not None:
            self._run_native(kind, x, y, b, omega, norm_out, dot_out)
            return
        if V.is_distributed and V.is_cart and not x._ghost_valid:
            # block decomposition: every decomposed axis' ghosts, then one launch
            V.dist.exchange(x._data, V.pads)
            x._ghost_valid = True
        n0 = V.local_npts[0] if V.ndim == 3 else 1
        st = _stream()
        ranges = ((0, n0, 0, 0),)
        handle = None
        if V.is_distributed and not x._ghost_valid:
            p0 = V.pads[0]
            handle = V.dist.start_exchange(V.planes(x._store), width=p0, pad=p0)
            if handle is not None and n0 > 2 * self.pmax:
                # interior planes meanwhile, then both p-plane boundaries in one launch
                ranges = ((self.pmax, n0 - self.pmax, 0, 0), (0, self.pmax, n0 - self.pmax, n0))
            else:
                V.dist.finish_exchange(handle)
                handle = None
        self._calls += 1
        epi = self._EPI[kind]
        xp, yp = rt.ptr(x._data), rt.ptr(y._data)
        bp = rt.ptr(b._data) if b is not None else None
        def _p(v):   # device tensor, raw device address (int) or None
            if v is None:
                return None
            return rt.ptr(v) if isinstance(v, torch.Tensor) else C.c_void_p(v)

        np_, dp = _p(norm_out), _p(dot_out)
        for idx, (zb, ze, zb2, ze2) in enumerate(ranges):
            if idx == 1 and handle is not None:
                V.dist.finish_exchange(handle)
                handle = None
            if self.timer is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            _lib.call("poms_op_run_reduce2", self._h, epi, float(omega), xp, yp, bp, zb, ze, zb2, ze2, np_, dp,
                      1 if idx else 0, st)
            if self.timer is not None:
                e1.record()
                self.timer.append((kind, e0, e1, self._calls))
        if handle is not None:
            V.dist.finish_exchange(handle)
        x._ghost_valid = True

    def _run_native(self, kind, x, y, b=None, omega=0.0, norm_out=None, dot_out=None, lazy_count=0,
                    host_dst=None):
        """The distributed call through the native communicator: exchange (if x's
        ghosts are stale), interior, both boundaries and the reductions in ONE host
        call (``poms_op_run_dist``).  With ``lazy_count`` returns the ticket of the
        all-reduced values being copied to ``host_dst``."""
        V = self.space
        d = V.dist
        st = _stream()
        self._calls += 1

        def _p(v):
            if v is None:
                return None
            return rt.ptr(v) if isinstance(v, torch.Tensor) else C.c_void_p(v)

        tk = C.c_int(-1)
        if self.timer is not None:   # per call: includes the wait for the exchange
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _lib.call("poms_op_run_dist", self._h, d.native.h, self._EPI[kind], float(omega), rt.ptr(x._data),
                  rt.ptr(y._data), rt.ptr(b._data) if b is not None else None,
                  C.c_void_p(V.planes(x._store).data_ptr()), V.plane_elems, V.local_npts[0], V.pads[0],
                  self.pmax, -1 if d.prev is None else d.prev, -1 if d.next is None else d.next,
                  0 if x._ghost_valid else 1, 1 if (norm_out is not None or (lazy_count and kind != "apply_dot"))
                  else 0, 1 if (dot_out is not None or (lazy_count == 2)) else 0, _p(norm_out), _p(dot_out),
                  int(lazy_count), C.c_void_p(host_dst.data_ptr()) if host_dst is not None else None,
                  C.byref(tk), st)
        if self.timer is not None:
            e1.record()
            self.timer.append((kind, e0, e1, self._calls))
        x._ghost_valid = True
        return tk.value

    def dot(self, x: StencilVector, out: StencilVector | None = None) -> StencilVector:
        """y = A x (spl ``StencilMatrix.dot``)."""
        self._check(x)
        y = self.space.empty() if out is None else out
        self._check(y)
        if y is x:
            raise ValueError("out must not alias x")

        self._run("apply", x, y)
        y._mark_written()
        return y

    @property
    def apply_dot_supported(self) -> bool:
        v = C.c_int()
        _lib.call("poms_op_apply_dot_supported", self._h, C.byref(v))
        return bool(v.value)

    def dot_inner(self, x: StencilVector, out: StencilVector, device: bool = False):
        """``out = A x`` and the global ``x . out`` from the same pass (pcg's q and p.q);
        with ``device`` the dot stays a device tensor of shape (1,)."""
        self._check(x, out)
        if out is x:
            raise ValueError("out must not alias x")
        V = self.space
        nb = V.scalar_buffer()
        self._run("apply_dot", x, out, dot_out=nb[4:5])
        out._mark_written()
        if device and V.lazy_reductions:
            return V.device_sum(nb[4:5])
        return V.global_dot(float(nb[4].item()))

    def residual(self, b: StencilVector, x: StencilVector, out: StencilVector | None = None) -> StencilVector:
        """r = b - A x, fused (`sources/solvers.py:85`, `sources/mg_jac.py:93`)."""
        self._check(b, x)
        r = self.space.empty() if out is None else out
        if r is x:
            raise ValueError("out must not alias x")

        self._run("residual", x, r, b=b)
        r._mark_written()
        return r

    @property
    def fused_dot_supported(self) -> bool:
        v = C.c_int()
        _lib.call("poms_op_fused_dot_supported", self._h, C.byref(v))
        return bool(v.value)

    def jacobi_sweep(self, b: StencilVector, x_in: StencilVector, x_out: StencilVector,
                     omega: float, want_norm: bool = False, want_dot: bool = False, lazy: bool = False,
                     device_dot: bool = False):
        """x_out = x_in + omega (b - A x_in)/diag(A).

        Returns the global ``||dr||^2`` (or None); with ``want_dot`` returns
        ``(||dr||^2 or None, x_out . b)``, the dot fused into the sweep.  With
        ``lazy`` (and ``want_norm``) the norm comes back as a :class:`LazyScalar`
        so the host can queue the next sweep before reading it.
        """
        self._check(b, x_in, x_out)
        if x_in is x_out:
            raise ValueError("x_out must not alias x_in")
        V = self.space
        nb = V.scalar_buffer()
        if lazy and want_norm and not want_dot and V.is_distributed and V.dist.native is not None:
            # native communicator: reduce into a host-mapped ring slot, summed over the
            # ranks on the host when read
            from .dist import LazyNative
            host = V.pinned_slots(1)
            ticket = self._run_native("jacobi", x_in, x_out, b, omega, lazy_count=1, host_dst=host)
            x_out._mark_written()
            return LazyNative(V.dist.native, ticket, host)
        self._run("jacobi", x_in, x_out, b=b, omega=omega, norm_out=nb[0:1] if want_norm else None,
                  dot_out=nb[4:5] if want_dot else None)
        x_out._mark_written()
        if want_dot and device_dot and not want_norm and V.lazy_reductions:
            return None, V.device_sum(nb[4:5])    # x_out . b as a device tensor (1,)
        if want_dot:
            host = nb.cpu()   # one read for both reductions
            nrm = V.global_dot(float(host[0])) if want_norm else None
            return nrm, V.global_dot(float(host[4]))
        if not want_norm:
            return None
        if lazy and V.lazy_reductions:
            return V.lazy_sum(nb[0:1])
        return V.global_dot(float(nb[0].item()))

    @property
    def from_zero_supported(self) -> bool:
        V = self.space
        if V.is_distributed and V.is_cart:
            # x1 = omega b / diag on the ghost rows of axes 1, 2 would need the
            # neighbours' diagonal: damped_jacobi forms x1 with diag_scale instead
            return False
        v = C.c_int()
        _lib.call("poms_op_from_zero_supported", self._h, C.byref(v))
        return bool(v.value)

    @property
    def sweep2_supported(self) -> bool:
        """Two sweeps per launch (``poms_op_sweep2_supported``): one-rank 2D p = 3."""
        if self.space.is_distributed:
            return False
        v = C.c_int()
        _lib.call("poms_op_sweep2_supported", self._h, C.byref(v))
        return bool(v.value)

    def jacobi_sweep2(self, b: StencilVector, x_in: StencilVector, x_out: StencilVector, omega: float,
                      want_norm: bool = False):
        """Damped-Jacobi sweeps k and k+1 from x_in in one launch; x_out = x_{k+1}
        (bitwise two :meth:`jacobi_sweep` calls).  Returns ``(||dr_k||^2,
        ||dr_{k+1}||^2)`` with ``want_norm``, else None."""
        self._check(b, x_in, x_out)
        if x_out is x_in or x_out is b:
            raise ValueError("x_out must not alias x_in or b")
        if not self.sweep2_supported:
            raise NotImplementedError("jacobi_sweep2: one-rank 2D p = 3 Kronecker operators only")
        nb = self.space.scalar_buffer()
        # norm_out <- ||dr_{k+1}||^2 (slot 1), dot_out <- ||dr_k||^2 (slot 0)
        self._run("sweep2", x_in, x_out, b=b, omega=omega, norm_out=nb[1:2] if want_norm else None,
                  dot_out=nb[0:1] if want_norm else None)
        x_out._mark_written()
        if not want_norm:
            return None
        host = nb.cpu()
        return float(host[0]), float(host[1])

    def jacobi3_from_zero(self, b: StencilVector, x_out: StencilVector, omega: float, want_norm: bool = False):
        """Damped-Jacobi sweeps 1-3 from x0 = 0 in one launch (``poms_op_jacobi3_from_zero``;
        the operators of :attr:`sweep2_supported`); x_out = x3.  Returns ``(||x1||^2,
        ||dr_2||^2, ||dr_3||^2)`` with ``want_norm``, else None."""
        self._check(b, x_out)
        if x_out is b:
            raise ValueError("x_out must not alias b")
        if not self.sweep2_supported:
            raise NotImplementedError("jacobi3_from_zero: one-rank 2D p = 3 Kronecker operators only")
        nb = self.space.scalar_buffer()
        _lib.call("poms_op_jacobi3_from_zero", self._h, float(omega), rt.ptr(b._data), rt.ptr(x_out._data),
                  rt.ptr(nb[0:3]) if want_norm else None, _stream())
        x_out._mark_written()
        if not want_norm:
            return None
        host = nb.cpu()
        return float(host[0]), float(host[1]), float(host[2])

    def jacobi_from_zero(self, b: StencilVector, x_out: StencilVector, omega: float,
                         want_norm: bool = False, lazy: bool = False):
        """Damped-Jacobi sweeps 1 and 2 from x0 = 0 in one pass over b; x_out = x2.

        Returns ``(||dr_1||^2, ||dr_2||^2)`` (floats), a :class:`LazyScalar` with
        those two values (``lazy``), or None without ``want_norm``.
        """
        self._check(b, x_out)
        if x_out is b:
            raise ValueError("x_out must not alias b")
        V = self.space
        if not self.from_zero_supported:
            raise NotImplementedError("jacobi_from_zero is not supported by this operator / decomposition")
        nb = V.scalar_buffer()
        if lazy and want_norm and V.is_distributed and V.dist.native is not None:
            from .dist import LazyNative
            host = V.pinned_slots(2)   # [||x1||^2, ||dr_2||^2]
            ticket = self._run_native("jacobi2", b, x_out, b, omega, lazy_count=2, host_dst=host)
            x_out._mark_written()
            return LazyNative(V.dist.native, ticket, host)
        # norm_out <- ||dr_2||^2 (slot 1), dot_out <- ||x1||^2 (slot 0): adjacent, one copy
        self._run("jacobi2", b, x_out, b=b, omega=omega, norm_out=nb[1:2] if want_norm else None,
                  dot_out=nb[0:1] if want_norm else None)
        x_out._mark_written()
        if not want_norm:
            return None
        if lazy and V.lazy_reductions:
            return V.lazy_sum(nb[0:2])
        host = nb.cpu()
        return V.global_dot(float(host[0])), V.global_dot(float(host[1]))

    def diag_scale(self, b: StencilVector, out: StencilVector, scale: float = 1.0, want_norm: bool = False,
                   lazy: bool = False):
        """out = scale * b / diag(A); returns global ||out||^2 or None."""
        self._check(b, out)
        V = self.space
        st = _stream()
        _lib.call("poms_op_diag_scale", self._h, float(scale), rt.ptr(b._data), rt.ptr(out._data),
                  int(want_norm), st)
        out._mark_written()
        if not want_norm:
            return None
        cnt = C.c_int64()
        _lib.call("poms_op_last_partials", self._h, C.byref(cnt))
        nb = V.scalar_buffer()
        _lib.call("poms_reduce_partials", V.ctx, cnt.value, rt.ptr(nb), st)
        if lazy and V.lazy_reductions:
            return V.lazy_sum(nb[0:1])
        return V.global_dot(float(nb[0].item()))

    # -- host-side views of the operator (set-up / API parity) --------------------
    def diagonal_axes(self):
        """Per-axis 1D diagonals of the global factors, by role name."""
        P = self.pmax
        return {k: v[:, P].copy() for k, v in self.bands.items()}

    def __getitem__(self, key):
        """Stencil entry ``A[i1, i2(, i3), k1, k2(, k3)]`` (global indices, offsets in [-p, p])."""
        nd = self.space.ndim
        if not isinstance(key, tuple) or len(key) != 2 * nd:
            raise IndexError("expected (i..., k...) with one index and one offset per axis")
        idx, off = key[:nd], key[nd:]
        P = self.pmax

        def ent(name, axis_rows_key, i, k):
            b = self.bands[name]
            if not 0 <= P + k < b.shape[1]:
                return 0.0
            return b[0 if b.shape[0] == 1 else i, P + k]

        if self.form == "sum":
            if nd == 3:
                return (ent("A0", 0, idx[0], off[0]) * ent("A1", 1, idx[1], off[1]) * ent("M2", 2, idx[2], off[2])
                        + ent("M0", 0, idx[0], off[0]) * (ent("B1", 1, idx[1], off[1]) * ent("M2", 2, idx[2], off[2])
                                                          + ent("A1", 1, idx[1], off[1]) * ent("K2", 2, idx[2], off[2])))
            if nd == 2:
                return (ent("A1", 1, idx[0], off[0]) * ent("M2", 2, idx[1], off[1])
                        + ent("B1", 1, idx[0], off[0]) * ent("K2", 2, idx[1], off[1]))
            return ent("A1", 1, 0, 0) * ent("M2", 2, idx[0], off[0]) + ent("B1", 1, 0, 0) * ent("K2", 2, idx[0], off[0])
        if nd == 3:
            return ent("F0", 0, idx[0], off[0]) * ent("F1", 1, idx[1], off[1]) * ent("F2", 2, idx[2], off[2])
        if nd == 2:
            return ent("F1", 1, idx[0], off[0]) * ent("F2", 2, idx[1], off[1])
        return ent("F2", 2, idx[0], off[0])

    def tosparse(self):
        """Global sparse matrix (small sizes; tests and coarse-grid set-up)."""
        import scipy.sparse as sp
        from .splines import band_to_dense
        D = {k: sp.csr_matrix(band_to_dense(v)) if v.shape[0] > 1 else sp.csr_matrix(v[:, self.pmax:self.pmax + 1])
             for k, v in self.bands.items()}
        nd = self.space.ndim
        kr = lambda *ms: _kron_all(ms)
        if self.form == "sum":
            if nd == 3:
                return kr(D["A0"], D["A1"], D["M2"]) + kr(D["M0"], D["B1"], D["M2"]) + kr(D["M0"], D["A1"], D["K2"])
            return kr(D["A1"], D["M2"]) + kr(D["B1"], D["K2"])
        if nd == 3:
            return kr(D["F0"], D["F1"], D["F2"])
        return kr(D["F1"], D["F2"])


def _kron_all(ms):
    import scipy.sparse as sp
    out = ms[0]
    for m in ms[1:]:
        out = sp.kron(out, m, format="csr")
    return out.tocsr()


class StencilMatrix(KronOperator):
    """spl ``StencilMatrix(V, W=None)`` with its own coefficients per row
    (`slides/content.tex:285-290`): ``v[i] = Σ_k M[i, k] u[i + k]``, ``k ∈ [-p, p]^d``.

    ``_data`` is the host array in spl's layout (padded local rows, then the
    ``2p+1`` offsets per axis); it is filled by ``M[i1, i2, k1, k2] = value`` (global
    row indices, slices allowed) exactly as the reference's ``assembly_2d`` does
    (`sources/matrix_assembler.py:84-179`), or from an assembled array with
    :meth:`from_data`.  The coefficients go to the device (``poms_op_create_stencil``)
    on the first device use after a change.  Every solver of :mod:`poms_amd.solvers`
    accepts it as ``A`` (general-stencil kernel, ``csrc/stencil_general.hip``)."""

    def __init__(self, V: StencilVectorSpace, W: StencilVectorSpace | None = None):
        if W is not None and W is not V:
            raise NotImplementedError("rectangular stencil matrices are not supported")
        self.space, self.form = V, "stencil"
        self.pmax = max(max(V.pads), 1)
        self.bands = {}
        self.timer = None
        self._calls = 0
        self._hh = C.c_void_p()
        self._dirty = True
        self._host = np.zeros(V.padded_shape + tuple(2 * p + 1 for p in V.pads))
        self.pads = V.pads
        self.starts, self.ends = V.starts, V.ends

    @classmethod
    def _from_handle(cls, V: StencilVectorSpace, h: C.c_void_p) -> "StencilMatrix":
        """Wrap a device-built general-stencil operator (``poms_op_assemble_stencil``);
        the host copy is fetched on first host-side access."""
        M = cls.__new__(cls)
        M.space, M.form = V, "stencil"
        M.pmax = max(max(V.pads), 1)
        M.bands, M.timer, M._calls = {}, None, 0
        M._hh, M._dirty, M._host = h, False, None
        M.pads, M.starts, M.ends = V.pads, V.starts, V.ends
        return M

    @property
    def _data(self) -> np.ndarray:
        """Host coefficients in the spl layout (downloaded once if device-built)."""
        if self._host is None:
            V = self.space
            out = np.zeros(V.padded_shape + tuple(2 * p + 1 for p in V.pads))
            _lib.call("poms_op_stencil_data", self._hh, out.ctypes.data_as(C.c_void_p))
            self._host = out
        return self._host

    @classmethod
    def from_data(cls, V: StencilVectorSpace, data: np.ndarray) -> "StencilMatrix":
        M = cls(V)
        data = np.asarray(data, dtype=np.float64)
        if data.shape != M._data.shape:
            raise ValueError(f"stencil data must have the spl shape {M._data.shape}")
        M._data[...] = data
        return M

    # the device handle, (re)created lazily after host-side changes
    @property
    def _h(self):
        if self._dirty:
            self._upload()
        return self._hh

    @_h.setter
    def _h(self, v):
        self._hh = v if v is not None else C.c_void_p()

    def _upload(self):
        V = self.space
        if self._hh.value:
            _lib.lib.poms_op_destroy(self._hh)
            self._hh = C.c_void_p()
        data = np.ascontiguousarray(self._data)
        h = C.c_void_p()
        g0 = V.starts[0] if V.ndim == 3 else 0
        n0g = V.npts[0] if V.ndim == 3 else 1
        _lib.call("poms_op_create_stencil", V.ctx, V.ndim, C.byref(V.layout), data.ctypes.data_as(C.c_void_p),
                  g0, n0g, C.byref(h))
        self._hh = h
        self._dirty = False

    def __del__(self):
        h = getattr(self, "_hh", None)
        if h is not None and h.value:
            try:
                _lib.lib.poms_op_destroy(h)
            except Exception:
                pass
            self._hh = C.c_void_p()

    # -- spl element access ----------------------------------------------------------
    def _idx(self, key):
        nd = self.space.ndim
        if not isinstance(key, tuple) or len(key) != 2 * nd:
            raise IndexError("expected (i..., k...) with one index and one offset per axis")
        out = []
        for d, (i, p, s) in enumerate(zip(key[:nd], self.pads, self.starts)):
            if isinstance(i, slice):
                if i != slice(None):
                    a = (i.start if i.start is not None else s) - s + p
                    b = (i.stop if i.stop is not None else self.ends[d] + 1) - s + p
                    out.append(slice(a, b))
                else:
                    out.append(slice(p, p + self.space.local_npts[d]))
            else:
                out.append(int(i) - s + p)
        for k, p in zip(key[nd:], self.pads):
            if isinstance(k, slice):
                out.append(slice((k.start if k.start is not None else -p) + p,
                                 (k.stop if k.stop is not None else p + 1) + p))
            else:
                out.append(int(k) + p)
        return tuple(out)

    def __getitem__(self, key):
        return self._data[self._idx(key)]

    def __setitem__(self, key, value):
        self._data[self._idx(key)] = value
        self._dirty = True

    def remove_spurious_entries(self):
        """Zero the coefficients that couple to points outside the (non-periodic) grid."""
        V = self.space
        nd = V.ndim
        for d in range(nd):
            p = self.pads[d]
            g = np.arange(V.local_npts[d]) + self.starts[d]
            for k in range(-p, p + 1):
                bad = (g + k < 0) | (g + k >= V.npts[d])
                if bad.any():
                    idx = [slice(None)] * (2 * nd)
                    idx[d] = np.nonzero(bad)[0] + p
                    idx[nd + d] = k + p
                    self._data[tuple(idx)] = 0.0
        self._dirty = True

    def tosparse(self):
        """Global sparse matrix of the local rows (small sizes)."""
        import scipy.sparse as sp
        V = self.space
        nd = V.ndim
        rows, cols, vals = [], [], []
        W = [2 * p + 1 for p in self.pads]
        inner = self._data[tuple(slice(p, p + n) for p, n in zip(self.pads, V.local_npts))]
        grid = np.stack(np.meshgrid(*[np.arange(n) + s for n, s in zip(V.local_npts, self.starts)],
                                    indexing="ij"), axis=-1).reshape(-1, nd)
        flat = inner.reshape(-1, int(np.prod(W)))
        for kk, ks in enumerate(np.ndindex(*W)):
            off = np.array(ks) - np.array(self.pads)
            tgt = grid + off
            ok = np.all((tgt >= 0) & (tgt < np.array(V.npts)), axis=1) & (flat[:, kk] != 0.0)
            rows.append(np.ravel_multi_index(grid[ok].T, V.npts))
            cols.append(np.ravel_multi_index(tgt[ok].T, V.npts))
            vals.append(flat[ok, kk])
        n = V.dimension
        return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))

    def tocsr(self):
        return self.tosparse()

    def toarray(self):
        return self.tosparse().toarray()

    def diagonal_axes(self):
        raise NotImplementedError("a general stencil has no per-axis factors")

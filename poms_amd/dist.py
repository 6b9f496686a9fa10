"""Slab decomposition along axis 0 and the p-plane ghost exchange.

The reference decomposes every axis with an MPI Cartesian topology (spl
``Cart``; ``sources/tests/test_kron_dot.py:51-55``) and exchanges ghost slabs
with subarray ``Irecv/Isend/Waitall`` per direction
(``pyccel/kron_product.py:21-41``).  On one MI355X node the natural
decomposition is 1D slabs of contiguous axis-0 planes, one rank per GPU: a
ghost region is then ``p`` whole padded planes -- contiguous in C order, so no
packing -- exchanged with rank +-1 by one grouped send/recv pair per side
(``torch.distributed.batch_isend_irecv`` = ``ncclGroupStart; ncclSend;
ncclRecv; ncclGroupEnd`` with the ``nccl``/RCCL backend over xGMI).

Split rule (matches spl's ``Cart`` block split): ``n`` planes over ``w`` ranks,
the first ``n % w`` ranks get one extra plane (515 = 3x65 + 5x64).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch


def slab_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Global ``[start, end)`` of ``rank``'s slab of ``n`` planes."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    size = base + (1 if rank < extra else 0)
    return start, start + size


@dataclass
class SlabDistribution:
    """Axis-0 slab of a global grid owned by ``rank`` out of ``world`` ranks."""

    n0_global: int
    rank: int
    world: int
    group: object = None
    cuda_transport: bool = True
    # global sums stay on the device (device tensors all-reduced by the backend);
    # default: with the RCCL transport.  gloo also reduces CUDA tensors (host
    # staged), which the 2-rank GPU test uses to run the device-scalar pcg path.
    device_reductions: bool | None = None

    def __post_init__(self):
        if self.device_reductions is None:
            self.device_reductions = self.cuda_transport
        self.native = None   # poms_comm handle (NativeComm) when the RCCL path is native
        self.start, self.end = slab_bounds(self.n0_global, self.world, self.rank)
        if self.end <= self.start:
            raise ValueError(f"rank {self.rank} owns no planes ({self.n0_global} over {self.world})")
        self.prev = self.rank - 1 if self.rank > 0 else None
        self.next = self.rank + 1 if self.rank + 1 < self.world else None

    @property
    def n_local(self) -> int:
        return self.end - self.start

    @classmethod
    def from_process_group(cls, n0_global: int, group=None, device_reductions: bool | None = None,
                           host_transport: bool = False, host_shm: bool = False) -> "SlabDistribution":
        """Slab of this rank.  With the ``nccl`` (RCCL) backend the library's own
        communicator is used (``POMS_NATIVE_COMM=0`` selects torch.distributed
        instead); if it cannot be created or fails its self-test this RAISES --
        a silent fall-back would hide a broken production path.  ``host_transport``
        (any backend, e.g. gloo): the same native schedule with the data moved by
        torch.distributed host callbacks (``poms_comm_create_host``); ``host_shm``
        adds the node-local shared-memory block for the host-read sums, the path
        every lazily read norm takes in a one-node RCCL run."""
        import torch.distributed as dist
        backend = dist.get_backend(group)
        d = cls(n0_global, dist.get_rank(group), dist.get_world_size(group), group,
                cuda_transport=(backend == "nccl"), device_reductions=device_reductions)
        if host_transport:
            if d.device_reductions is None or not d.device_reductions:
                d.device_reductions = True
            d.native = NativeComm.create_host(group, shm=host_shm)
        elif backend == "nccl" and d.world > 1 and os.environ.get("POMS_NATIVE_COMM", "1") != "0":
            d.native = NativeComm.create(group)
        return d

    @classmethod
    def loopback(cls, n0_global: int, rank: int, world: int) -> "SlabDistribution":
        """Rank ``rank``'s slab of a ``world``-rank split, run ALONE on this GPU, its
        halo exchanges and sums going through a one-rank RCCL communicator: every
        exchange sends the slab's boundary planes to itself (the ghosts then hold the
        slab's own planes, not a neighbour's) and every all-reduce is a one-rank RCCL
        call.  A timing proxy for one rank of the N-GPU run (``tools/slab_proxy.py``):
        that rank's kernels, exchanges and sums on the production schedule, with
        RCCL's on-device copy in place of the xGMI transfer.  Its results are not
        the global problem's."""
        d = cls(n0_global, rank, world, None, cuda_transport=True, device_reductions=True)
        d.native = NativeComm.create_loopback()
        d.prev = 0 if d.prev is not None else None   # the communicator's only rank
        d.next = 0 if d.next is not None else None
        return d

    @property
    def transport(self) -> str:
        """Which path moves ghosts and sums: "native" (RCCL from C), "native-host"
        (the C schedule over host callbacks), "native-loopback" (:meth:`loopback`),
        "torch" (torch.distributed) or "none"."""
        if self.world == 1:
            return "none"
        if self.native is None:
            return "torch"
        if self.native.is_loopback:
            return "native-loopback"
        return "native-host" if self.native.is_host else "native"

    # ------------------------------------------------------------------
    def start_exchange(self, data: torch.Tensor, width: int, pad: int):
        """Begin the axis-0 ghost exchange of a padded local array.

        ``data`` has shape ``(n_local + 2*pad, ...)``.  The first / last
        ``width`` owned planes go to the previous / next rank and the
        neighbours' planes land in this rank's ghost planes.  Returns a handle
        for :meth:`finish_exchange`.  Global-boundary ghosts stay untouched
        (zero: non-periodic, spurious band entries removed -- ``sources/utils.py:16``).
        """
        import torch.distributed as dist
        if width > pad:
            raise ValueError("ghost width exceeds storage pad")
        if width == 0 or (self.prev is None and self.next is None):
            return None
        n = self.n_local
        if n < width:
            raise ValueError(f"slab of {n} planes is thinner than the ghost width {width}")
        if self.native is not None:
            from . import runtime as rt
            # ranks of the native communicator are the group's ranks
            self.native.halo_start(data, n, pad, width, -1 if self.prev is None else self.prev,
                                   -1 if self.next is None else self.next, rt.stream_handle())
            return ("native",)
        staged = not self.cuda_transport and data.device.type != "cpu"
        buf = data.cpu() if staged else data
        ops, recv_views = [], []
        if self.prev is not None:
            lo_send = buf[pad:pad + width]
            lo_recv = buf[pad - width:pad] if not staged else torch.empty_like(buf[pad - width:pad])
            ops.append(dist.P2POp(dist.isend, lo_send.contiguous() if staged else lo_send,
                                  self._peer(self.prev), self.group))
            ops.append(dist.P2POp(dist.irecv, lo_recv, self._peer(self.prev), self.group))
            recv_views.append((slice(pad - width, pad), lo_recv))
        if self.next is not None:
            hi_send = buf[pad + n - width:pad + n]
            hi_recv = buf[pad + n:pad + n + width] if not staged else torch.empty_like(buf[pad + n:pad + n + width])
            ops.append(dist.P2POp(dist.isend, hi_send.contiguous() if staged else hi_send,
                                  self._peer(self.next), self.group))
            ops.append(dist.P2POp(dist.irecv, hi_recv, self._peer(self.next), self.group))
            recv_views.append((slice(pad + n, pad + n + width), hi_recv))
        works = dist.batch_isend_irecv(ops)
        return (works, staged, data, recv_views)

    def finish_exchange(self, handle) -> None:
        if handle is None:
            return
        if handle[0] == "native":
            from . import runtime as rt
            self.native.halo_finish(rt.stream_handle())
            return
        works, staged, data, recv_views = handle
        for w in works:
            w.wait()
        if staged:
            for sl, t in recv_views:
                data[sl].copy_(t)

    def exchange(self, data: torch.Tensor, width: int, pad: int) -> None:
        self.finish_exchange(self.start_exchange(data, width, pad))

    def _peer(self, r: int) -> int:
        if self.group is None:
            return r
        import torch.distributed as dist
        return dist.get_global_rank(self.group, r)


def dims_create(world: int, ndim: int) -> tuple[int, ...]:
    """Balanced process grid of ``world`` ranks over ``ndim`` axes, non-increasing
    (``MPI_Dims_create``'s rule, which spl's ``Cart`` uses when the caller gives
    no grid): prime factors, largest first, each to the currently smallest axis."""
    if world < 1 or ndim < 1:
        raise ValueError("bad world/ndim")
    f, n, q = [], world, 2
    while q * q <= n:
        while n % q == 0:
            f.append(q)
            n //= q
        q += 1
    if n > 1:
        f.append(n)
    dims = [1] * ndim
    for q in sorted(f, reverse=True):
        dims[dims.index(min(dims))] *= q
    return tuple(sorted(dims, reverse=True))


class CartDistribution:
    """Block decomposition of every axis over a process grid (spl ``Cart``).

    The reference builds ``Cart(npts, pads, periods, reorder, comm)``
    (`sources/tests/test_kron_dot.py:51-55, 89-93`; `slides/content.tex:200-223`):
    a Cartesian communicator whose rank owns the block ``[starts[d], ends[d]]`` of
    each axis and exchanges ``pads[d]``-wide ghost layers with its two neighbours
    along every decomposed axis.  Here: ranks in C order over ``dims`` (rank =
    ((c0 d1) + c1) d2 + c2, MPI_Cart_create without reordering), each axis split
    as :func:`slab_bounds`, and :meth:`exchange` fills the ghost layers axis by
    axis -- axis d's faces span the full padded extents of the other axes, so the
    edge and corner ghosts arrive through the later axes (the same scheme as
    spl's per-direction subarray exchange, `pyccel/kron_product.py:21-41`).

    The slab decomposition (:class:`SlabDistribution`) is the ``dims = (w, 1, 1)``
    case with the native RCCL schedule; this general grid moves its faces with
    ``torch.distributed`` (RCCL device-to-device with ``nccl``, host-staged with
    gloo) and one blocking exchange per operator call.
    """

    native = None   # no native communicator: faces move through torch.distributed

    def __init__(self, npts, dims, rank: int, group=None, cuda_transport: bool = True,
                 device_reductions: bool | None = None):
        self.npts = tuple(int(n) for n in npts)
        self.dims = tuple(int(d) for d in dims)
        self.ndim = len(self.npts)
        if len(self.dims) != self.ndim or any(d < 1 for d in self.dims):
            raise ValueError("dims must give one positive grid extent per axis")
        self.world = int(np.prod(self.dims))
        if not 0 <= rank < self.world:
            raise ValueError(f"rank {rank} outside a grid of {self.world}")
        self.rank, self.group = int(rank), group
        self.cuda_transport = cuda_transport
        self.device_reductions = cuda_transport if device_reductions is None else device_reductions
        self.coords = self.coords_of(self.rank)
        b = [slab_bounds(n, d, c) for n, d, c in zip(self.npts, self.dims, self.coords)]
        self.starts = tuple(s for s, _ in b)
        self.ends = tuple(e for _, e in b)   # exclusive
        for d, (s, e) in enumerate(b):
            if e <= s:
                raise ValueError(f"axis {d}: rank {rank} owns no points ({self.npts[d]} over {self.dims[d]})")
        self.prev = tuple(self.rank_of(self._shift(d, -1)) if self.coords[d] > 0 else None
                          for d in range(self.ndim))
        self.next = tuple(self.rank_of(self._shift(d, 1)) if self.coords[d] + 1 < self.dims[d] else None
                          for d in range(self.ndim))

    def coords_of(self, rank: int) -> tuple[int, ...]:
        out = []
        for d in reversed(self.dims):
            out.append(rank % d)
            rank //= d
        return tuple(reversed(out))

    def rank_of(self, coords) -> int:
        r = 0
        for c, d in zip(coords, self.dims):
            r = r * d + c
        return r

    def _shift(self, axis: int, step: int):
        c = list(self.coords)
        c[axis] += step
        return c

    @property
    def n_local(self) -> tuple[int, ...]:
        return tuple(e - s for s, e in zip(self.starts, self.ends))

    @property
    def transport(self) -> str:
        return "none" if self.world == 1 else "torch"

    @classmethod
    def from_process_group(cls, npts, dims=None, group=None,
                           device_reductions: bool | None = None) -> "CartDistribution":
        """Block of this rank; ``dims`` defaults to :func:`dims_create`."""
        import torch.distributed as dist
        world = dist.get_world_size(group)
        dims = dims_create(world, len(npts)) if dims is None else tuple(dims)
        if int(np.prod(dims)) != world:
            raise ValueError(f"process grid {dims} does not hold {world} ranks")
        return cls(npts, dims, dist.get_rank(group), group, cuda_transport=(dist.get_backend(group) == "nccl"),
                   device_reductions=device_reductions)

    def _peer(self, r: int) -> int:
        if self.group is None:
            return r
        import torch.distributed as dist
        return dist.get_global_rank(self.group, r)

    def exchange(self, data: torch.Tensor, pads, widths=None) -> None:
        """Fill the ghost layers of the padded local block ``data`` (shape
        ``n_local[d] + 2 pads[d]`` per axis; strided views allowed) from the
        neighbours, ``widths[d]`` (default ``pads[d]``) layers per decomposed axis.
        Ghosts past the global boundary are left untouched (zero)."""
        import torch.distributed as dist
        nd = self.ndim
        widths = tuple(pads) if widths is None else tuple(widths)
        staged = not self.cuda_transport and data.device.type != "cpu"
        for ax in range(nd):
            if self.dims[ax] == 1 or widths[ax] == 0:
                continue
            w, p, n = widths[ax], pads[ax], self.n_local[ax]
            if w > p:
                raise ValueError("ghost width exceeds storage pad")
            if n < w:
                raise ValueError(f"axis {ax}: block of {n} points is thinner than the ghost width {w}")

            def face(lo, hi):
                idx = [slice(None)] * nd
                idx[ax] = slice(lo, hi)
                return data[tuple(idx)]

            ops, recvs = [], []
            for nbr, send, ghost in ((self.prev[ax], face(p, p + w), face(p - w, p)),
                                     (self.next[ax], face(p + n - w, p + n), face(p + n, p + n + w))):
                if nbr is None:
                    continue
                sbuf = send.contiguous()
                if staged:
                    sbuf = sbuf.cpu()
                rbuf = torch.empty(ghost.shape, dtype=data.dtype, device="cpu" if staged else data.device)
                ops.append(dist.P2POp(dist.isend, sbuf, self._peer(nbr), self.group))
                ops.append(dist.P2POp(dist.irecv, rbuf, self._peer(nbr), self.group))
                recvs.append((ghost, rbuf))
            if ops:
                for wk in dist.batch_isend_irecv(ops):
                    wk.wait()
            for ghost, rbuf in recvs:
                ghost.copy_(rbuf)


class NativeComm:
    """The library's own RCCL communicator over the process group's ranks
    (``poms_comm_*``, ``csrc/comm.hip``): ghost exchanges and scalar all-reduces
    cost the host one C call each instead of a torch.distributed round trip.

    :meth:`create` runs a self-test (an all-reduce and a ghost exchange checked
    against their known results, both run on every rank before either is judged)
    and RAISES if it fails on any rank; ``POMS_NATIVE_COMM=0`` selects the
    torch.distributed transport explicitly.

    ``POMS_COMM_PEER=1`` (the same on every rank) moves the ghost exchange to the
    peer transport (``poms_comm_set_peer``): one kernel of ``POMS_PEER_WGS``
    (default 32) workgroups that stores the boundary planes into the neighbours'
    IPC-mapped mailboxes -- no RCCL call, capturable.  The self-test then runs it."""

    def __init__(self, handle, device: int, callbacks=None):
        import ctypes as C
        from . import _lib
        self.h = handle
        self.device = device
        self._callbacks = callbacks   # host transport: keep the ctypes thunks alive
        self.is_loopback = False
        s = C.c_void_p()
        _lib.call("poms_comm_stream", self.h, C.byref(s))
        self.stream = torch.cuda.ExternalStream(s.value, device=torch.device("cuda", device))
        yes = C.c_int()
        _lib.call("poms_comm_is_host", self.h, C.byref(yes))
        self.is_host = bool(yes.value)
        self.peer = False
        if os.environ.get("POMS_COMM_PEER", "0") == "1":
            self.set_peer(True)

    def set_peer(self, enable: bool, wgs: int | None = None) -> None:
        """Peer transport for the ghost exchange on (every rank alike) or off; ``wgs``
        exchange workgroups (default ``POMS_PEER_WGS``, else 32: equal on every rank,
        which the mailbox set-up checks)."""
        from . import _lib
        if wgs is None:
            wgs = int(os.environ.get("POMS_PEER_WGS", "32"))
        _lib.call("poms_comm_set_peer", self.h, 1 if enable else 0, int(wgs))
        self.peer = bool(enable)

    def peer_reserve(self, cnt: int, prev: int, nxt: int) -> None:
        """Build the peer mailboxes for exchanges of up to ``cnt`` doubles per side now
        (collective with the two neighbours), not at the first such exchange -- which
        may be inside a graph capture."""
        from . import _lib
        _lib.call("poms_comm_peer_reserve", self.h, int(cnt), int(prev), int(nxt))

    def peer_status(self) -> dict:
        """{"active", "fine_grained", "timed_out"} of the peer transport (synchronises
        the communication stream)."""
        import ctypes as C
        from . import _lib
        a, f, t = C.c_int(), C.c_int(), C.c_int()
        _lib.call("poms_comm_peer_status", self.h, C.byref(a), C.byref(f), C.byref(t))
        return {"active": bool(a.value), "fine_grained": bool(f.value), "timed_out": bool(t.value)}

    def check(self) -> None:
        """Raise if a peer exchange of this communicator timed out (its ghosts, and
        everything computed from them, are invalid); no synchronisation."""
        from . import _lib
        _lib.call("poms_comm_check", self.h)

    @property
    def uses_shm(self) -> bool:
        """The lazily read sums go through the node-local shared-memory block."""
        import ctypes as C
        from . import _lib
        yes = C.c_int()
        _lib.call("poms_comm_uses_shm", self.h, C.byref(yes))
        return bool(yes.value)

    @classmethod
    def create(cls, group=None):
        """RCCL communicator over the group's ranks, self-tested; raises on failure."""
        import ctypes as C
        import torch.distributed as dist
        from . import _lib
        dev = torch.cuda.current_device()
        nb = _lib.lib.poms_comm_id_bytes()
        obj = [None]
        if dist.get_rank(group) == 0:
            buf = C.create_string_buffer(nb)
            _lib.call("poms_comm_unique_id", buf, nb)
            obj[0] = bytes(buf.raw[:nb])
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        h = C.c_void_p()
        _lib.call("poms_comm_create", dev, C.c_char_p(obj[0]), dist.get_rank(group),
                  dist.get_world_size(group), C.byref(h))
        comm = cls(h, dev)
        comm._check_self_test(group)
        return comm

    @classmethod
    def create_loopback(cls):
        """A one-rank RCCL communicator on the current GPU (no process group); see
        :meth:`SlabDistribution.loopback`."""
        import ctypes as C
        from . import _lib
        dev = torch.cuda.current_device()
        nb = _lib.lib.poms_comm_id_bytes()
        buf = C.create_string_buffer(nb)
        _lib.call("poms_comm_unique_id", buf, nb)
        h = C.c_void_p()
        _lib.call("poms_comm_create", dev, buf, 0, 1, C.byref(h))
        comm = cls(h, dev)
        comm.is_loopback = True
        return comm

    @classmethod
    def create_host(cls, group=None, shm: bool = False):
        """The native schedule over torch.distributed host callbacks (any backend).

        The C side stages the boundary planes / scalars through host memory and
        calls back: the exchange is one ``batch_isend_irecv`` with rank +-1 on CPU
        tensors, the sum one ``all_reduce``.  Used by the multi-rank tests to drive
        ``poms_op_run_dist``'s schedule with real neighbours where RCCL cannot run
        (several ranks on one GPU).  ``shm``: attach the node-local shared-memory
        block (``poms_comm_host_attach_shm``, id broadcast from rank 0) so that the
        lazily read sums run ``shm_allsum`` as in a one-node RCCL run; raises if
        the ranks do not all find each other in it."""
        import ctypes as C
        import numpy as np
        import torch.distributed as dist
        from . import _lib

        def peer(r):
            return r if group is None else dist.get_global_rank(group, r)

        def view(ptr, cnt):
            return torch.from_numpy(np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_double)), shape=(int(cnt),)))

        def exchange(user, slo, rlo, shi, rhi, cnt, prev, nxt):
            try:
                ops = []
                if prev >= 0:
                    ops.append(dist.P2POp(dist.isend, view(slo, cnt), peer(prev), group))
                    ops.append(dist.P2POp(dist.irecv, view(rlo, cnt), peer(prev), group))
                if nxt >= 0:
                    ops.append(dist.P2POp(dist.isend, view(shi, cnt), peer(nxt), group))
                    ops.append(dist.P2POp(dist.irecv, view(rhi, cnt), peer(nxt), group))
                if ops:
                    for w in dist.batch_isend_irecv(ops):
                        w.wait()
                return 0
            except Exception:   # reported through poms_last_error by the caller
                return 1

        def allreduce(user, buf, cnt):
            try:
                dist.all_reduce(view(buf, cnt), group=group)
                return 0
            except Exception:
                return 1

        XF = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                         C.c_int, C.c_int)
        AF = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64)
        cbs = (XF(exchange), AF(allreduce))
        dev = torch.cuda.current_device()
        h = C.c_void_p()
        _lib.call("poms_comm_create_host", dev, dist.get_rank(group), dist.get_world_size(group),
                  C.cast(cbs[0], C.c_void_p), C.cast(cbs[1], C.c_void_p), None, C.byref(h))
        comm = cls(h, dev, callbacks=cbs)
        if shm and dist.get_world_size(group) > 1:
            obj = [os.urandom(32) if dist.get_rank(group) == 0 else None]
            dist.broadcast_object_list(obj, src=peer(0), group=group)
            att = C.c_int()
            _lib.call("poms_comm_host_attach_shm", comm.h, C.c_char_p(obj[0]), len(obj[0]), C.byref(att))
            if not att.value:
                raise RuntimeError("host transport: the node-local shared-memory block was not attached on every rank")
        comm._check_self_test(group)
        return comm

    def _check_self_test(self, group):
        """All ranks agree that the all-reduce and the ghost exchange work, or raise."""
        import torch.distributed as dist
        try:
            ok = self._self_test(dist.get_rank(group), dist.get_world_size(group))
            err = ""
        except Exception as e:
            ok, err = False, repr(e)
        oks = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
        if dist.get_backend(group) == "nccl":
            oks = oks.to(f"cuda:{self.device}")
        dist.all_reduce(oks, op=dist.ReduceOp.MIN, group=group)
        if float(oks.item()) < 1.0:
            raise RuntimeError(f"native communicator failed its self-test on some rank {err}".strip())

    def _self_test(self, rank: int, world: int) -> bool:
        from . import runtime as rt
        dev = f"cuda:{self.device}"
        t = torch.full((2,), float(rank + 1), dtype=torch.float64, device=dev)
        self.allreduce(t, rt.stream_handle(), wait_back=True)
        # judged only after the exchange below: a rank that returned here would leave its
        # neighbours blocked in their halo_start, and the job would hang instead of raising
        ok = bool(torch.allclose(t.cpu(), torch.full((2,), world * (world + 1) / 2.0, dtype=torch.float64)))
        pad, width, n_loc, pe = 2, 2, 3, 8
        data = torch.zeros((n_loc + 2 * pad, pe), dtype=torch.float64, device=dev)
        for i in range(n_loc):
            data[pad + i] = 1000.0 * rank + i
        prev = rank - 1 if rank > 0 else -1
        nxt = rank + 1 if rank + 1 < world else -1
        self.halo_start(data, n_loc, pad, width, prev, nxt, rt.stream_handle())
        self.halo_finish(rt.stream_handle())
        # one round of the host-read sums (the damped-Jacobi / pcg stop tests): the
        # rank's value goes straight into a ring slot (pinned host memory, the same
        # address on the host), the wait adds the ranks' values on the host -- through
        # the node-local shared-memory block when attached (one-node RCCL runs)
        import ctypes as C
        addr, ticket = self.slot()
        vals = (C.c_double * 2).from_address(addr)
        vals[0], vals[1] = float(rank + 1), float(2 * rank + 1)
        host_slot = torch.zeros(2, dtype=torch.float64)
        lz = self.to_host(ticket, 2, host_slot, rt.stream_handle())
        s0, s1 = lz.value(0), lz.value(1)
        ok = ok and s0 == world * (world + 1) / 2.0 and s1 == float(world * world)
        h = data.cpu()
        if self.peer and self.peer_status()["timed_out"]:
            return False
        for j in range(width):
            lo = h[pad - width + j]   # planes n_loc-width+j of rank-1
            hi = h[pad + n_loc + j]   # planes j of rank+1
            if prev >= 0 and not bool((lo == 1000.0 * prev + (n_loc - width + j)).all()):
                return False
            if prev < 0 and bool(lo.any()):
                return False
            if nxt >= 0 and not bool((hi == 1000.0 * nxt + j).all()):
                return False
            if nxt < 0 and bool(hi.any()):
                return False
        return ok

    def halo_start(self, data: torch.Tensor, n_local: int, pad: int, width: int, prev: int, nxt: int, stream):
        from . import _lib
        import ctypes as C
        _lib.call("poms_halo_start", self.h, C.c_void_p(data.data_ptr()), int(data.stride(0)), int(n_local),
                  int(pad), int(width), int(prev), int(nxt), stream)

    def halo_finish(self, stream):
        from . import _lib
        _lib.call("poms_halo_finish", self.h, stream)

    def slot(self):
        """(device address, ticket) of the next ring slot (2 doubles) for a lazily
        read global sum."""
        from . import _lib
        import ctypes as C
        p, t = C.c_void_p(), C.c_int()
        _lib.call("poms_comm_slot", self.h, C.byref(p), C.byref(t))
        return p.value, t.value

    def to_host(self, ticket: int, count: int, host_slot: torch.Tensor, stream) -> "LazyNative":
        """Ring slot ``ticket`` is written by the launch just queued on ``stream``; the
        returned object's ``value(i)`` waits for it, sums it over the ranks on the host
        (``poms_comm_wait``) and reads the global sum from ``host_slot``."""
        from . import _lib
        import ctypes as C
        _lib.call("poms_allreduce_to_host", self.h, int(ticket), int(count), C.c_void_p(host_slot.data_ptr()),
                  stream)
        return LazyNative(self, ticket, host_slot)

    def allreduce(self, t: torch.Tensor, stream, wait_back: bool):
        from . import _lib
        import ctypes as C
        self.check()
        _lib.call("poms_allreduce_sum", self.h, C.c_void_p(t.data_ptr()), int(t.numel()), stream,
                  1 if wait_back else 0)


class LazyNative:
    """A global sum of the native communicator's host-side ring (the LazyScalar
    interface): ``value`` waits for the launch's local sum and adds the ranks' sums
    on the host."""

    def __init__(self, comm: NativeComm, ticket: int, host_slot: torch.Tensor):
        self._comm, self._ticket, self._host = comm, ticket, host_slot
        self._done = False

    def value(self, i: int = 0) -> float:
        if not self._done:
            from . import _lib
            _lib.call("poms_comm_wait", self._comm.h, self._ticket)
            self._done = True
        return float(self._host[i])

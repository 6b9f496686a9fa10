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

from dataclasses import dataclass

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
        self.start, self.end = slab_bounds(self.n0_global, self.world, self.rank)
        if self.end <= self.start:
            raise ValueError(f"rank {self.rank} owns no planes ({self.n0_global} over {self.world})")
        self.prev = self.rank - 1 if self.rank > 0 else None
        self.next = self.rank + 1 if self.rank + 1 < self.world else None

    @property
    def n_local(self) -> int:
        return self.end - self.start

    @classmethod
    def from_process_group(cls, n0_global: int, group=None, device_reductions: bool | None = None
                           ) -> "SlabDistribution":
        import torch.distributed as dist
        backend = dist.get_backend(group)
        return cls(n0_global, dist.get_rank(group), dist.get_world_size(group), group,
                   cuda_transport=(backend == "nccl"), device_reductions=device_reductions)

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

"""Device plumbing: one libpoms_hip context per GPU, torch streams, communicator.

PyTorch is used only for device memory, streams and ``torch.distributed``
(RCCL over xGMI when the process group backend is ``nccl``).  All arithmetic
on the hot path goes through ``libpoms_hip.so``; nothing here computes.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import torch

from . import _lib

_CTX: dict[int, C.c_void_p] = {}


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("poms_amd needs a ROCm GPU (gfx950): torch.cuda.is_available() is False")


def device_index(device=None) -> int:
    require_gpu()
    if device is None:
        return torch.cuda.current_device()
    return torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()


def ctx(dev: int) -> C.c_void_p:
    """libpoms_hip context of device ``dev`` (created once per process)."""
    h = _CTX.get(dev)
    if h is None:
        h = C.c_void_p()
        _lib.call("poms_ctx_create", dev, C.byref(h))
        _CTX[dev] = h
    return h


def stream_handle() -> C.c_void_p:
    """hipStream_t of torch's current stream (kernels are ordered with torch ops).

    Uses torch's raw-stream query (the public ``current_stream()`` costs ~8 us of
    host time per call, which the V-cycle makes ~700 times)."""
    try:
        return C.c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))
    except AttributeError:   # older torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


@dataclass
class Comm:
    """Thin wrapper of a torch.distributed process group (None = single rank)."""

    group: object = None
    enabled: bool = False
    cuda_transport: bool = False  # nccl (= RCCL on ROCm) moves device tensors

    @classmethod
    def from_env(cls, group=None) -> "Comm":
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return cls()
        backend = dist.get_backend(group)
        return cls(group=group, enabled=dist.get_world_size(group) > 1,
                   cuda_transport=(backend == "nccl"))

    @property
    def rank(self) -> int:
        import torch.distributed as dist
        return dist.get_rank(self.group) if self.enabled else 0

    @property
    def size(self) -> int:
        import torch.distributed as dist
        return dist.get_world_size(self.group) if self.enabled else 1

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum across ranks (RCCL on device tensors, else staged via host)."""
        if not self.enabled:
            return t
        import torch.distributed as dist
        if self.cuda_transport or t.device.type == "cpu":
            dist.all_reduce(t, group=self.group)
        else:
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        return t

    def allreduce_scalar(self, v: float) -> float:
        """Sum of one double over the ranks (a device tensor for RCCL: nccl has no CPU path)."""
        if not self.enabled:
            return v
        dev = torch.device("cuda", torch.cuda.current_device()) if self.cuda_transport else torch.device("cpu")
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        import torch.distributed as dist
        dist.all_reduce(t, group=self.group)
        return float(t.item())


def sqrt(v: float) -> float:
    return math.sqrt(v)

#!/usr/bin/env python3
"""Round 6: the library's RCCL ghost exchange under hipGraph capture, with capture driven
from the HIP C API (ctypes) instead of torch.cuda.graph (round-5 verdict item 4).

tools/r06/graph_probe.cpp showed that RCCL's grouped self send / receive captures and
replays correctly from the C API -- on the capturing stream, on a forked stream, on a
forked highest-priority stream, in global and relaxed mode, with RCCL 2.27.7 (ROCm) and
2.26.6 (torch's) alike.  This probe runs the LIBRARY's exchange (poms_halo_start /
poms_halo_finish on a one-rank loopback communicator: events, the communication stream,
grouped ncclSend / ncclRecv) the same way, each stage in a process of its own:

  capi          hipStreamBeginCapture (relaxed) / EndCapture / hipGraphInstantiate
                (flags 0) / 3 replays, every return code checked, ghosts compared with
                the eager exchange
  capi_autofree the same, instantiated with hipGraphInstantiateFlagAutoFreeOnLaunch
  capi_torchst  capi on a torch.cuda.Stream (torch's capture stream type)
  torch         torch.cuda.graph(capture_error_mode="relaxed"), as round 5 (crashed there)
  capi_onepeer  capi on the loopback of rank 0 of 4 (one neighbour side: ONE send /
                receive pair in the group; rank 1's loopback has both sides = rank 0)

    python tools/r06/graph_probe_lib.py --stages capi,capi_autofree,capi_torchst,torch
"""
from __future__ import annotations

import argparse
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def _setup(cells=40, p=3, rank=1, world=4):
    import torch
    from poms_amd.dist import SlabDistribution
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    n = cells + p
    d = SlabDistribution.loopback(n, rank, world)
    M, K = assemble_1d(uniform_knots(p, cells), p)
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True, dist=d)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    return torch, d, V, A


def _hip():
    h = C.CDLL("libamdhip64.so")
    for name, args in {"hipStreamBeginCapture": [C.c_void_p, C.c_int],
                       "hipStreamEndCapture": [C.c_void_p, C.POINTER(C.c_void_p)],
                       "hipGraphGetNodes": [C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t)],
                       "hipGraphInstantiateWithFlags": [C.c_void_p, C.c_void_p, C.c_ulonglong],
                       "hipGraphLaunch": [C.c_void_p, C.c_void_p],
                       "hipStreamSynchronize": [C.c_void_p],
                       "hipStreamCreateWithFlags": [C.POINTER(C.c_void_p), C.c_uint],
                       "hipGetErrorString": [C.c_int]}.items():
        getattr(h, name).argtypes = args
        getattr(h, name).restype = C.c_int if name != "hipGetErrorString" else C.c_char_p
    return h


def _ck(h, rc, what):
    if rc != 0:
        raise SystemExit(f"FAIL {what}: {h.hipGetErrorString(rc).decode()} ({rc})")
    print(f"  step: {what}", flush=True)


def run(stage: str):
    torch, d, V, A = _setup(rank=0 if stage == "capi_onepeer" else 1)
    from poms_amd import _lib
    x = V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    planes = V.planes(x._store)
    pad = V.pads[0]
    prev = -1 if d.prev is None else d.prev
    nxt = -1 if d.next is None else d.next
    h = _hip()
    if stage == "capi_torchst" or stage == "torch":
        ts = torch.cuda.Stream()
        sptr = ts.cuda_stream
    else:
        s = C.c_void_p()
        _ck(h, h.hipStreamCreateWithFlags(C.byref(s), 1), "hipStreamCreateWithFlags(non-blocking)")
        sptr = s.value

    def exch():
        _lib.call("poms_halo_start", d.native.h, C.c_void_p(planes.data_ptr()), V.plane_elems, V.local_npts[0], pad,
                  pad, prev, nxt, C.c_void_p(sptr))
        _lib.call("poms_halo_finish", d.native.h, C.c_void_p(sptr))

    exch()
    _ck(h, h.hipStreamSynchronize(C.c_void_p(sptr)), "eager exchange")
    ref = x._store.clone()
    planes[:pad].zero_()
    planes[-pad:].zero_()
    torch.cuda.synchronize()
    if stage == "torch":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=ts, capture_error_mode="relaxed"):
            exch()
        print("  step: torch capture_end returned", flush=True)
        for _ in range(3):
            g.replay()
    else:
        _ck(h, h.hipStreamBeginCapture(C.c_void_p(sptr), 2), "hipStreamBeginCapture(relaxed)")   # 2 = relaxed
        exch()
        print("  step: exchange queued in capture", flush=True)
        graph = C.c_void_p()
        _ck(h, h.hipStreamEndCapture(C.c_void_p(sptr), C.byref(graph)), "hipStreamEndCapture")
        nn = C.c_size_t(0)
        _ck(h, h.hipGraphGetNodes(graph, None, C.byref(nn)), "hipGraphGetNodes")
        print(f"  captured graph: {nn.value} nodes", flush=True)
        if nn.value == 0:
            raise SystemExit("FAIL: nothing captured")
        ge = C.c_void_p()
        flags = 1 if stage == "capi_autofree" else 0   # hipGraphInstantiateFlagAutoFreeOnLaunch
        _ck(h, h.hipGraphInstantiateWithFlags(C.byref(ge), graph, flags), f"hipGraphInstantiateWithFlags({flags})")
        for _ in range(3):
            _ck(h, h.hipGraphLaunch(ge, C.c_void_p(sptr)), "hipGraphLaunch")
        _ck(h, h.hipStreamSynchronize(C.c_void_p(sptr)), "replays done")
    torch.cuda.synchronize()
    assert torch.equal(x._store, ref), "captured exchange != eager exchange"
    print(f"{stage} ok", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="capi,capi_autofree,capi_torchst,torch")
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        import faulthandler
        faulthandler.enable()
        run(a.child)
        return 0
    for s in a.stages.split(","):   # each stage in its own process; stop at the first crash
        r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, "--child", s], capture_output=True, text=True,
                           timeout=180)
        tail = "\n".join((r.stdout + r.stderr).strip().splitlines()[-25:])
        print(f"=== stage {s}: exit {r.returncode}\n{tail}\n", flush=True)
        if r.returncode < 0 or r.returncode in (124, 134, 137, 139):
            print("crash / abort: stopping", flush=True)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Which part of a distributed smoother call breaks hipGraph capture? (round-4 verdict
item 2: `POMS_PCG_GRAPH=2 tools/slab_proxy.py --loopback-rank 1` dumped core.)

Each stage runs in a child process with faulthandler on, so a crash names its stage
and the Python frame that made the native call; the parent prints every stage's exit
status and stderr tail:

  halo      one ghost exchange (grouped ncclSend/ncclRecv on the communication
            stream, ordered by events) captured with torch.cuda.graph, replayed 3x,
            ghosts checked against the eager exchange;
  allreduce one in-place ncclAllReduce captured and replayed;
  split     one distributed Jacobi sweep (poms_op_run_dist: exchange, interior
            launch, boundary launch on the communication stream, device sums)
            captured and replayed, checked bitwise against the eager call;
  pcg       pcg + damped Jacobi in speculative mode replayed from the library's own
            captured graph (POMS_PCG_SPEC=1 POMS_PCG_GRAPH=2) against the
            step-by-step loop, on rank 1 of an 8-rank split looped back.

    python tools/graph_rccl_probe.py [--stages halo,allreduce,split,pcg]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
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


def stage_halo():
    import ctypes as C
    torch, d, V, A = _setup()
    from poms_amd import _lib
    x = V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    st = torch.cuda.Stream()
    planes = V.planes(x._store)
    pad = V.pads[0]

    def exch(s):
        _lib.call("poms_halo_start", d.native.h, C.c_void_p(planes.data_ptr()), V.plane_elems, V.local_npts[0], pad,
                  pad, -1 if d.prev is None else d.prev, -1 if d.next is None else d.next, C.c_void_p(s.cuda_stream))
        _lib.call("poms_halo_finish", d.native.h, C.c_void_p(s.cuda_stream))

    with torch.cuda.stream(st):
        exch(st)
    torch.cuda.synchronize()
    ref = x._store.clone()
    planes[:pad].zero_()
    planes[-pad:].zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st, capture_error_mode="relaxed"):
        exch(st)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(x._store, ref), "captured exchange != eager exchange"
    print("halo ok", flush=True)


def stage_allreduce():
    import ctypes as C
    torch, d, V, A = _setup()
    from poms_amd import _lib
    buf = torch.arange(8, dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st, capture_error_mode="relaxed"):
        _lib.call("poms_allreduce_sum", d.native.h, C.c_void_p(buf.data_ptr()), 8, C.c_void_p(st.cuda_stream), 1)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(buf.cpu(), torch.arange(8, dtype=torch.float64)), "one-rank all-reduce changed the values"
    print("allreduce ok", flush=True)


def stage_split():
    torch, d, V, A = _setup()
    x, b = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    y_ref, y = V.zeros(), V.zeros()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        x._ghost_valid = False
        A.jacobi_sweep(b, x, y_ref, 2.0 / 3.0, want_norm=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st, capture_error_mode="relaxed"):
        x._ghost_valid = False   # the exchange, interior, boundary launch on the comm stream
        A.jacobi_sweep(b, x, y, 2.0 / 3.0, want_norm=False)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y._store, y_ref._store), "captured sweep != eager sweep"
    print("split ok", flush=True)


def stage_pcg():
    torch, d, V, A = _setup(cells=48, rank=1, world=4)
    from poms_amd import solvers
    b = V.zeros()
    V.interior(b._data).fill_(1.0)
    out = {}
    for mode in ("step", "graph"):
        os.environ["POMS_PCG_SPEC"] = "1" if mode == "graph" else "0"
        os.environ["POMS_PCG_GRAPH"] = "2" if mode == "graph" else "0"
        for rep in range(3):   # the graph run captures once, then replays
            x, info = solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=4)
        torch.cuda.synchronize()
        out[mode] = (x._data.clone(), dict(info))
    assert out["step"][1] == out["graph"][1], (out["step"][1], out["graph"][1])
    assert torch.equal(out["step"][0], out["graph"][0]), "graph replay != step-by-step loop"
    st = A.spec_stats if hasattr(A, "spec_stats") else None
    print("pcg ok", out["graph"][1], "spec stats", st, flush=True)


STAGES = {"halo": stage_halo, "allreduce": stage_allreduce, "split": stage_split, "pcg": stage_pcg}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="allreduce,halo,split,pcg")
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        import faulthandler
        faulthandler.enable()
        STAGES[a.child]()
        return 0
    bad = False
    for s in a.stages.split(","):   # every stage, each in its own process
        r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, "--child", s], capture_output=True, text=True,
                           timeout=240)
        tail = "\n".join((r.stdout + r.stderr).strip().splitlines()[-25:])
        print(f"=== stage {s}: exit {r.returncode}\n{tail}\n", flush=True)
        bad = bad or r.returncode != 0
        if r.returncode < 0 or r.returncode in (124, 134, 137, 139):   # nothing more on the GPU after a crash
            print("crash / abort: stopping", flush=True)
            return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())

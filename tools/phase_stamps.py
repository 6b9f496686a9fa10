#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the fused kernel's plane loop (s_memtime
stamps, separate build).  Shares only -- stamps perturb the schedule."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

PHASES = ["xs_store", "barrier1", "prefetch_issue", "axis2", "barrier2", "axis1", "axis0", "epilogue"]


def main():
    import torch
    from poms_amd import _lib, runtime as rt
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, int(sys.argv[1]) if len(sys.argv) > 1 else 512
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * 3, [p] * 3)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x, b, y = V.zeros(), V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    for variant in (1, 2):
        A.set_variant(variant)
        for jac in (0, 1):
            dbg = torch.zeros(4 << 20, dtype=torch.int64, device="cuda")
            nw = C.c_int64()
            for _ in range(2):
                _lib.call("poms_op_profile_phases", A._h, jac, rt.ptr(b._data), rt.ptr(x._data),
                          rt.ptr(y._data), rt.ptr(dbg), C.byref(nw), rt.stream_handle())
            torch.cuda.synchronize()
            d = dbg[: nw.value * 8].view(nw.value, 8).double()
            tot = d.sum(0)
            share = (tot / tot.sum()).tolist()
            print(f"variant {variant} {'jacobi' if jac else 'apply '}: " +
                  " ".join(f"{ph}={s*100:.1f}%" for ph, s in zip(PHASES, share)), flush=True)


if __name__ == "__main__":
    main()

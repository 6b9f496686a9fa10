#!/usr/bin/env python3
"""Round 6: the ubench's memory-only march (tools/r06/ublib.hip, t16) on the library's own
515^3 arrays, interleaved in one process with the production v5 apply (variant 10) --
does the harness (allocation, layout) or the kernel make the v5 apply's memory pattern
slower than the ubench's?"""
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, 512
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x, y = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    assert tuple(x._data.stride()) == (521 * 528, 528, 1) and x._data.data_ptr() % 128 == 104, (x._data.stride(), x._data.data_ptr() % 128)
    ub = C.CDLL(str(ROOT / "tools/r06/ublib.so"))
    st = torch.cuda.current_stream()
    res = {}
    for rnd in range(3):
        for kind in ("v5", "ub", "ub_trim", "ub_fma64"):
            ts = []
            for _ in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind == "v5":
                    A.dot(x, out=y)
                else:
                    rc = ub.ub_t16(C.c_void_p(x._data.data_ptr()), C.c_void_p(y._data.data_ptr()),
                                   1 if kind != "ub" else 0, 64 if kind == "ub_fma64" else 0, C.c_void_p(st.cuda_stream))
                    assert rc == 0
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            res.setdefault(kind, []).extend(e0.elapsed_time(e1) * 1e3 for e0, e1 in ts[2:])
    for k, v in res.items():
        print(json.dumps({"kind": k, "median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1)}))


if __name__ == "__main__":
    main()

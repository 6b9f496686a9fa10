#!/usr/bin/env python3
"""Round-5 experiment: the v5 apply with one barrier per two planes (diagnostic
variant 115, CP bit 128 in kron_v5.hip: a 6-deep x ring, x(t+4) and x(t+5) DMA'd
after the barrier of every even plane) against the production apply (variant 10):
bitwise at several sizes, then interleaved timing at 515^3.

    python tools/r05/pb2_check.py [--cells 512] [--reps 20] [--rounds 6]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--variant", type=int, default=115)
    a = ap.parse_args()
    import torch
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace

    def make(cells, p=3, align=True):
        M, K = assemble_1d(uniform_knots(p, cells), p)
        n = cells + p
        V = StencilVectorSpace([n] * 3, [p] * 3, align=align)
        return V, KronOperator.laplace(V, [M] * 3, [K] * 3)

    bad = 0
    for cells, align in [(20, True), (45, False), (109, True), (200, True), (253, False), (512, True)]:
        V, A = make(cells, align=align)
        x = V.zeros()
        V.interior(x._data).uniform_(-1, 1, generator=torch.Generator(device="cuda").manual_seed(cells))
        ys = []
        for var in (10, a.variant):
            A.set_variant(var)
            y = V.zeros()
            A.dot(x, out=y)
            torch.cuda.synchronize()
            assert A.last_variant == var, (A.last_variant, var)
            ys.append(y._data.clone())
        eq = torch.equal(ys[0], ys[1])
        bad += not eq
        print(f"cells {cells} align {align}: variant {a.variant} == 10 bitwise: {eq}", flush=True)
        del V, A, x, ys
        torch.cuda.empty_cache()
    if bad:
        print("PARITY FAIL", flush=True)
        return 1
    V, A = make(a.cells)
    x, y = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    res = {10: [], a.variant: []}
    for rnd in range(a.rounds):
        for var in ((10, a.variant) if rnd % 2 == 0 else (a.variant, 10)):
            A.set_variant(var)
            for _ in range(3):
                A.dot(x, out=y)
            torch.cuda.synchronize()
            A.timer = []
            for _ in range(a.reps):
                A.dot(x, out=y)
            torch.cuda.synchronize()
            ts = [e0.elapsed_time(e1) * 1e3 for _, e0, e1, _c in A.timer]
            A.timer = None
            res[var] += ts
            print(f"  round {rnd} variant {var}: median {statistics.median(ts):.1f} min {min(ts):.1f} us", flush=True)
    for var, ts in res.items():
        print(f"variant {var}: apply median {statistics.median(ts):.1f} us min {min(ts):.1f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

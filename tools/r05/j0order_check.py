#!/usr/bin/env python3
"""Round-5 experiment: the two-sweeps-from-zero launch with its slow tile rows (off the
axis-1 Toeplitz interior) dispatched first (diagnostic variant 116, CP bit 256) against
the production order (variant 10): bitwise on several sizes (x2 and both norms), then
interleaved timing at 515^3.

    python tools/r05/j0order_check.py [--cells 512] [--reps 20]

Variant 116 exists only with profiles/r05/j0order/slowfirst.patch applied: bitwise
equal (sums included), median 770.3 against 763.8 us, so it was not kept.
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
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--rounds", type=int, default=4)
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
    for cells, align in [(20, True), (45, False), (109, True), (200, True), (253, False)]:
        V, A = make(cells, align=align)
        b = V.zeros()
        V.interior(b._data).uniform_(-1, 1)
        res = []
        for var in (10, 116):
            A.set_variant(var)
            y = V.zeros()
            nr = A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True)
            torch.cuda.synchronize()
            res.append((y._data.clone(), nr))
        eq = torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]
        bad += not eq
        print(f"cells {cells} align {align}: variant 116 == 10 bitwise (x2, norms): {eq} {res[0][1]} {res[1][1]}",
              flush=True)
    if bad:
        print("PARITY FAIL", flush=True)
        return 1
    V, A = make(a.cells)
    b, y = V.zeros(), V.zeros()
    V.interior(b._data).uniform_(-1, 1)
    res = {10: [], 116: []}
    for _ in range(a.rounds):
        for var in (10, 116):
            A.set_variant(var)
            for _ in range(2):
                A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=False)
            torch.cuda.synchronize()
            A.timer = []
            for _ in range(a.reps):
                A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=False)
            torch.cuda.synchronize()
            res[var] += [e0.elapsed_time(e1) * 1e3 for _, e0, e1, _c in A.timer]
            A.timer = None
    for var, ts in res.items():
        print(f"variant {var}: from_zero median {statistics.median(ts):.1f} us min {min(ts):.1f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

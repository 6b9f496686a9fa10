#!/usr/bin/env python3
"""Round-5 experiment: the v5 apply with its x rows read by inline asm and counted
LDS waits (diagnostic variant 115) against the production apply (variant 10):
bitwise equality on several sizes, both row layouts, then interleaved timing.

    python tools/r05/asmrd_check.py [--cells 512] [--reps 20]

Variant 115 exists only with profiles/r05/asmrd/asmrd_experiment.patch applied (it was
bitwise equal and 3 % slower: 546.0 vs 529.7 us, so it was not kept).
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
    for cells, align in [(20, True), (40, False), (109, True), (200, True), (253, False)]:
        V, A = make(cells, align=align)
        x = V.zeros()
        V.interior(x._data).uniform_(-1, 1)
        ys = []
        for var in (10, 115):
            A.set_variant(var)
            y = V.zeros()
            A.dot(x, out=y)
            torch.cuda.synchronize()
            ys.append(y._data.clone())
        eq = torch.equal(ys[0], ys[1])
        bad += not eq
        print(f"cells {cells} align {align}: variant 115 == 10 bitwise: {eq}"
              + ("" if eq else f" max |d| {(ys[0] - ys[1]).abs().max().item():.3e}"), flush=True)
    if bad:
        print("PARITY FAIL", flush=True)
        return 1

    V, A = make(a.cells)
    x, y = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    dof = (a.cells + 3) ** 3
    res = {10: [], 115: []}
    for _ in range(a.rounds):
        for var in (10, 115):
            A.set_variant(var)
            for _ in range(2):
                A.dot(x, out=y)
            torch.cuda.synchronize()
            A.timer = []
            for _ in range(a.reps):
                A.dot(x, out=y)
            torch.cuda.synchronize()
            res[var] += [e0.elapsed_time(e1) * 1e3 for _, e0, e1, _c in A.timer]
            A.timer = None
    for var, ts in res.items():
        med = statistics.median(ts)
        print(f"variant {var}: apply median {med:.1f} us min {min(ts):.1f} us  {16 * dof / med / 1e3:.0f} GB/s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

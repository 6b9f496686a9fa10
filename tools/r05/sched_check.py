#!/usr/bin/env python3
"""Round-5 check of the v5 dispatch order (KronGeom::sched, kron_v5.hip: each XCD
starts its tiles longest-estimated first; poms_diag_v5_sched toggles it).

1. Bitwise: apply, residual, Jacobi sweep + norm, two sweeps from zero + norms,
   apply + dot, at several sizes, with the order on and off.  The partial sums keep
   their default slots, so the norms must agree bitwise too.
2. Timing at 515^3: the same launches interleaved, order on / off, per round.

    python tools/r05/sched_check.py [--cells 512] [--reps 15] [--rounds 4]
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
    ap.add_argument("--kinds", default="from_zero,jacobi,apply")
    a = ap.parse_args()
    import torch
    from poms_amd import _lib
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace

    def sched(mode):
        return _lib.lib.poms_diag_v5_sched(mode)

    def make(cells, p=3, align=True):
        M, K = assemble_1d(uniform_knots(p, cells), p)
        n = cells + p
        V = StencilVectorSpace([n] * 3, [p] * 3, align=align)
        return V, KronOperator.laplace(V, [M] * 3, [K] * 3)

    bad = 0
    for cells, align in [(20, True), (45, False), (109, True), (200, True), (253, False)]:
        V, A = make(cells, align=align)
        A.set_variant(10)
        x, b = V.zeros(), V.zeros()
        g = torch.Generator(device="cuda").manual_seed(cells)
        V.interior(x._data).uniform_(-1, 1, generator=g)
        V.interior(b._data).uniform_(-1, 1, generator=g)
        res = []
        for mode in (0, 1):
            sched(mode)
            y, r, xo, j0 = V.zeros(), V.zeros(), V.zeros(), V.zeros()
            A.dot(x, out=y)
            A.residual(b, x, out=r)
            n1 = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
            n0 = A.jacobi_from_zero(b, j0, 2.0 / 3.0, want_norm=True)
            ad = float(A.dot_inner(x, V.zeros(), device=True))
            torch.cuda.synchronize()
            res.append(([t._data.clone() for t in (y, r, xo, j0)], (n1, n0, ad)))
        eq = all(torch.equal(u, v) for u, v in zip(res[0][0], res[1][0])) and res[0][1] == res[1][1]
        bad += not eq
        print(f"cells {cells} align {align}: order on == off bitwise (apply, residual, sweep, from zero, "
              f"norms, apply+dot): {eq} {res[0][1]} {res[1][1]}", flush=True)
    if bad:
        print("PARITY FAIL", flush=True)
        return 1

    V, A = make(a.cells)
    A.set_variant(10)
    x, b, y = V.zeros(), V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    fns = {"apply": lambda: A.dot(x, out=y),
           "jacobi": lambda: A.jacobi_sweep(b, x, y, 2.0 / 3.0, want_norm=False),
           "from_zero": lambda: A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=False)}
    for kind in a.kinds.split(","):
        fn = fns[kind]
        res = {0: [], 1: []}
        for rnd in range(a.rounds):
            for mode in ((0, 1) if rnd % 2 == 0 else (1, 0)):
                sched(mode)
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                A.timer = []
                for _ in range(a.reps):
                    fn()
                torch.cuda.synchronize()
                ts = [e0.elapsed_time(e1) * 1e3 for _, e0, e1, _c in A.timer]
                A.timer = None
                res[mode] += ts
                print(f"  {kind} round {rnd} order {'on ' if mode else 'off'}: median {statistics.median(ts):.1f} "
                      f"min {min(ts):.1f} us", flush=True)
        for mode, ts in res.items():
            print(f"{kind} order {'on ' if mode else 'off'}: median {statistics.median(ts):.1f} us min {min(ts):.1f} us "
                  f"({len(ts)} launches)", flush=True)
    sched(1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

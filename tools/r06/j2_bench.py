#!/usr/bin/env python3
"""Round 6: time the two-sweep launch (epilogue 6) against two single v3 sweeps on the
2D bench grid, with spline bands (Toeplitz interior: fast tiles) and random bands (every
tile on the per-row / per-lane band path), to see what bounds the launch."""
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def _rand(p, n, rng):
    M = rng.uniform(-1, 1, (n, 2 * p + 1))
    K = rng.uniform(-1, 1, (n, 2 * p + 1))
    M[:, p] += 4.0
    K[:, p] = np.abs(K[:, p]) + 1.0
    return M, K


def main():
    import torch
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p, N = 3, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n = N + p
    rng = np.random.default_rng(0)
    for kind in ("spline", "random"):
        F = [assemble_1d(uniform_knots(p, N), p) if kind == "spline" else _rand(p, n, rng) for _ in range(2)]
        V = StencilVectorSpace([n, n], [p, p], align=True)
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        b = V.zeros().from_numpy(rng.standard_normal((n, n)))
        x = V.zeros().from_numpy(rng.standard_normal((n, n)))
        y, z = V.zeros(), V.zeros()
        res = {}
        for name, fn in (("sweep", lambda: A.jacobi_sweep(b, x, y, 0.6)),
                         ("two_sweeps", lambda: (A.jacobi_sweep(b, x, y, 0.6), A.jacobi_sweep(b, y, z, 0.6))),
                         ("sweep2", lambda: A.jacobi_sweep2(b, x, y, 0.6))):
            for _ in range(5):
                fn()
            ts = []
            for _ in range(40):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            t = [a.elapsed_time(c) * 100.0 for a, c in ts]   # us per call
            res[name] = round(statistics.median(t), 2)
        print(f"{kind} {n}^2: us per call (queued back to back)", res, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

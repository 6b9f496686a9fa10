#!/usr/bin/env python3
"""Round 6: is the two-sweep launch's bad tile deterministic?  Repeats and seeds."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    for cells in ((150, 130), (130, 150), (100, 200), (200, 100)):
        F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
        n = [N + p for N in cells]
        V = StencilVectorSpace(n, [p, p])
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        for seed in (0, 1):
            rng = np.random.default_rng(seed)
            b = V.zeros().from_numpy(rng.standard_normal(n))
            x0 = V.zeros().from_numpy(rng.standard_normal(n))
            x1, x2 = V.zeros(), V.zeros()
            A.jacobi_sweep(b, x0, x1, 2.0 / 3.0)
            A.jacobi_sweep(b, x1, x2, 2.0 / 3.0)
            r = x2._data.cpu().numpy()
            for rep in range(3):
                y = V.zeros()
                A.jacobi_sweep2(b, x0, y, 2.0 / 3.0)
                torch.cuda.synchronize()
                a = y._data.cpu().numpy()
                d = np.abs(a - r)
                bad = np.argwhere(d > 0)
                ti = {}
                for i, j in bad:
                    key = (int((i - p) // 48), int((j - p) // 52))
                    ti.setdefault(key, []).append((int(i), int(j)))
                desc = {k: (len(v), min(x[0] for x in v), max(x[0] for x in v), min(x[1] for x in v),
                            max(x[1] for x in v)) for k, v in sorted(ti.items())}
                print(f"cells {cells} seed {seed} rep {rep}: bad {len(bad)} tiles {desc}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

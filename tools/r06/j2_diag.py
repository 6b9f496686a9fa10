#!/usr/bin/env python3
"""Round 6: where the two-sweep launch (epilogue 6) differs from two single sweeps."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    for cells in ((64, 64), (150, 130), (7, 9)):
        p = 3
        rng = np.random.default_rng(sum(cells))
        F = [assemble_1d(uniform_knots(p, N), p) for N in cells]
        n = [N + p for N in cells]
        V = StencilVectorSpace(n, [p, p])
        A = KronOperator.laplace(V, [f[0] for f in F], [f[1] for f in F])
        b = V.zeros().from_numpy(rng.standard_normal(n))
        x0 = V.zeros().from_numpy(rng.standard_normal(n))
        x1, x2, y = V.zeros(), V.zeros(), V.zeros()
        om = 2.0 / 3.0
        n1 = A.jacobi_sweep(b, x0, x1, om, want_norm=True)
        n2 = A.jacobi_sweep(b, x1, x2, om, want_norm=True)
        m1, m2 = A.jacobi_sweep2(b, x0, y, om, want_norm=True)
        a, r = y._data.cpu().numpy(), x2._data.cpu().numpy()
        d = np.abs(a - r)
        bad = np.argwhere(d > 0)
        print(f"cells {cells}: storage {a.shape}, norms k {n1:.17g} vs {m1:.17g}, k+1 {n2:.17g} vs {m2:.17g}")
        print(f"  mismatches {len(bad)}, max abs {d.max():.3e}, max |ref| {np.abs(r).max():.3e}")
        if len(bad):
            rows = sorted(set(bad[:, 0].tolist()))
            cols = sorted(set(bad[:, 1].tolist()))
            print("  rows", rows[:40], "... n", len(rows))
            print("  cols", cols[:70], "... n", len(cols))
            for i, j in bad[:10]:
                print(f"   ({i},{j}) got {a[i, j]:.17g} want {r[i, j]:.17g}")
        T, TO = 48, 52
        ti = {}
        for i, j in bad:
            key = ((i - p) // T, (j - p) // TO)
            ti[key] = max(ti.get(key, 0.0), d[i, j])
        print("  per tile (t1, t2): max abs diff", {k: f"{v:.2e}" for k, v in sorted(ti.items())})
        big = np.argwhere(d > 1e-10)
        if len(big):
            print("  big rows", sorted(set(big[:, 0].tolist()))[:60])
            print("  big cols", sorted(set(big[:, 1].tolist()))[:80])
    return 0


if __name__ == "__main__":
    sys.exit(main())

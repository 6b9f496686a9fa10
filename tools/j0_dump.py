#!/usr/bin/env python3
"""Two sweeps from zero on a fixed random right-hand side: writes the output and
both norms to an .npz (compare two libraries through POMS_HIP_LIB)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    out, cells = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    p = 3
    M, K = assemble_1d(uniform_knots(p, cells), p)
    n = cells + p
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    b = V.zeros().from_numpy(np.random.default_rng(7).standard_normal((n,) * 3))
    y = V.zeros()
    m1, m2 = A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True)
    np.savez(out, y=y.to_local_numpy(), m1=m1, m2=m2, variant=A.kernel_variant("jacobi_from_zero"))
    print(out, m1, m2)


if __name__ == "__main__":
    main()

"""Locate mismatches between the v5 apply (variant 10) and v3 (variant 9) at full size."""
import sys
import torch
sys.path.insert(0, ".")
from poms_amd.splines import assemble_1d, uniform_knots
from poms_amd.stencil import KronOperator, StencilVectorSpace

p, N = int(sys.argv[1]), int(sys.argv[2])
align = len(sys.argv) > 3 and sys.argv[3] == "align"
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 10
M, K = assemble_1d(uniform_knots(p, N), p)
n = N + p
V = StencilVectorSpace([n] * 3, [p] * 3, align=align)
A = KronOperator.laplace(V, [M] * 3, [K] * 3)
x = V.zeros()
g = torch.Generator(device="cuda").manual_seed(1)
V.interior(x._data).uniform_(-1, 1, generator=g)
x._mark_written()
A.set_variant(9)
ref = V.interior(A.dot(x)._data).clone()
A.set_variant(variant)
print("variant", variant, "p", p, "N", N, "align", align)
for rep in range(6):
    y = V.interior(A.dot(x)._data)
    d = (y - ref).abs() > 1e-12 * ref.abs().max()
    print("rep", rep, "bad", int(d.sum()), "of", d.numel())
    if d.any():
        w = d.nonzero()[0]
        print("  first bad: got", float(y[tuple(w)]), "want", float(ref[tuple(w)]),
              "x there", float(V.interior(x._data)[tuple(w)]))
    if d.any():
        idx = d.nonzero()
        for ax in range(3):
            u, c = torch.unique(idx[:, ax], return_counts=True)
            print("  axis", ax, "values", u[:20].tolist(), "counts", c[:20].tolist(), "nuniq", len(u))

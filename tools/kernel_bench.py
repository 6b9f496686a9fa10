#!/usr/bin/env python3
"""Micro-benchmark of the fused Kronecker kernels (apply / residual / Jacobi sweep).

Interleaves variants (chunk sizes, kernel variants) in ONE process, reporting
median / min per-launch time from HIP events on the launch stream and the
algorithmic GB/s (apply 16 B/DOF, residual and Jacobi 24 B/DOF).

    python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --chunks 0,32,64
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=512)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--ndim", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--chunks", type=str, default="0")
    ap.add_argument("--tile-cols", type=str, default="0", help="comma list of v3/v4 output columns per tile")
    ap.add_argument("--no-align", action="store_true", help="unpadded row pitch (n2 + 2p)")
    ap.add_argument("--variants", type=str, default="")
    ap.add_argument("--kinds", type=str, default="apply,jacobi")
    ap.add_argument("--json", type=str, default="")
    ap.add_argument("--dump", action="store_true", help="print every launch time (us) of each row")
    ap.add_argument("--flush", action="store_true",
                    help="write a 512 MiB buffer before every timed launch (evicts L2 and the 256 MiB MALL)")
    a = ap.parse_args()

    import torch
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace

    p, N, nd = a.p, a.cells, a.ndim
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * nd, [p] * nd, align=not a.no_align)
    A = KronOperator.laplace(V, [M] * nd, [K] * nd)
    x, b, y = V.zeros(), V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    dof = n ** nd
    flush = torch.zeros(64 << 20, dtype=torch.float64, device="cuda") if a.flush else None
    chunks = [int(c) for c in a.chunks.split(",")]
    tile_cols = [int(c) for c in a.tile_cols.split(",")]
    variants = [int(v) for v in a.variants.split(",")] if a.variants else [None]
    kinds = a.kinds.split(",")
    res = {}
    for rnd in range(a.rounds):
        for ch, tcols in [(c, t) for c in chunks for t in tile_cols]:
            A.set_chunk(ch)
            A.set_tile_cols(tcols)
            for var in variants:
                if var is not None:
                    A.set_variant(var)
                for kind in kinds:
                    fn = {"dot": lambda: x.dot(b),
                          "apply": lambda: A.dot(x, out=y),
                          "apply_dot": lambda: A.dot_inner(x, y, device=True),
                          "residual": lambda: A.residual(b, x, out=y),
                          "jacobi": lambda: A.jacobi_sweep(b, x, y, 2.0 / 3.0, want_norm=False),
                          "from_zero": lambda: A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=False)}[kind]
                    for _ in range(2):
                        fn()
                    torch.cuda.synchronize()
                    A.timer = []
                    ev = []
                    for _ in range(a.reps):
                        if flush is not None:
                            flush.add_(1.0)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        fn()
                        e1.record()
                        ev.append((e0, e1))
                    torch.cuda.synchronize()
                    if A.timer:   # per-launch kernel events (operator kinds)
                        ts = [e0.elapsed_time(e1) * 1e3 for _, e0, e1, _c in A.timer]
                    else:         # whole call (dot includes its reduction + host read)
                        ts = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
                    A.timer = None
                    res.setdefault((ch, tcols, var, kind), []).extend(ts)
    out = []
    for (ch, tcols, var, kind), ts in res.items():
        med = statistics.median(ts)
        bpd = 16 if kind in ("apply", "apply_dot", "dot", "from_zero") else 24
        row = {"chunk": ch, "tile_cols": tcols, "aligned": not a.no_align, "variant": var, "kind": kind, "median_us": med, "min_us": min(ts),
               **({"launch_us": [round(t, 1) for t in ts]} if a.dump else {}),
               "GBps": bpd * dof / med / 1e3, "GDOFps": dof / med / 1e3}
        out.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

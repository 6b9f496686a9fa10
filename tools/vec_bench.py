#!/usr/bin/env python3
"""Timing of pcg's flat vector updates at the bench size (515^3, p = 3, aligned):
r -= alpha q with r.r partials (RUPD, 24 B/DOF) and x += alpha p, p = s + beta p
(XPUPD, 40 B/DOF), device coefficients, HIP events around each launch.

    POMS_VEC_BLOCKS=2048 python tools/vec_bench.py --reps 30
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=512)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from poms_amd import solvers
    from poms_amd.stencil import StencilVectorSpace
    n = a.cells + a.p
    V = StencilVectorSpace([n] * 3, [a.p] * 3, align=True)
    vs = [V.zeros() for _ in range(5)]
    for v in vs:
        V.interior(v._data).uniform_(-1, 1)
    x, p, s, r, q = vs
    ab = torch.tensor([1e-3, 0.5], dtype=torch.float64, device="cuda")
    fns = {"rupd": lambda: solvers._pcg_r_update_dev(V, ab[0:1], r, q),
           "xpupd": lambda: solvers._pcg_xp_update_dev(V, ab, x, p, s)}
    out = {}
    for name, fn in fns.items():
        for _ in range(3):
            fn()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        us = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ts]
        bpd = 24 if name == "rupd" else 40
        med = statistics.median(us)
        out[name] = {"median_us": round(med, 1), "min_us": round(min(us), 1), "TBps": round(bpd * n ** 3 / med / 1e6, 3)}
    print(json.dumps({"blocks": os.environ.get("POMS_VEC_BLOCKS", "4096"), **out}), flush=True)


if __name__ == "__main__":
    main()

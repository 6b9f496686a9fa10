#!/usr/bin/env python3
"""Residual -> restriction, fused (one pass over x and b) against the unfused pair
(residual vector, then restriction), plus the prolong-add, at a bench size; and the
V-cycle with and without the fused pass, interleaved.  Medians of HIP-event timings."""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=3)
    ap.add_argument("--cells", type=int, default=512)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cycles", type=int, default=4)
    a = ap.parse_args()
    import torch
    from poms_amd.mg import TwoLevelVCycle
    torch.cuda.set_device(0)
    mg = TwoLevelVCycle(a.p, a.cells, 8, ndim=a.ndim)
    A, tr, V = mg.A, mg.transfer, mg.space
    bf = mg.rhs_ones()
    x = V.zeros()
    torch.manual_seed(0)
    V.interior(x._data).uniform_(-1, 1)
    r = V.empty()

    def med(fn):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        return round(ts[len(ts) // 2], 1)

    out = {"ndim": a.ndim, "cells": a.cells, "p": a.p, "dof": V.dimension}
    for _ in range(2):
        tr.resid_restrict(A, bf, x, out=mg.rc)
        tr.restrict(A.residual(bf, x, out=r), out=mg.rc)
    out["fused_us"] = med(lambda: tr.resid_restrict(A, bf, x, out=mg.rc))
    out["residual_us"] = med(lambda: A.residual(bf, x, out=r))
    out["restrict_us"] = med(lambda: tr.restrict(r, out=mg.rc))
    out["prolong_add_us"] = med(lambda: tr.prolong_add(mg.xc, x))
    out["fused_GBps_16BperDOF"] = round(16 * V.dimension / out["fused_us"] / 1e3, 1)
    out["prolong_GBps_16BperDOF"] = round(16 * V.dimension / out["prolong_add_us"] / 1e3, 1)
    # V-cycle A/B, interleaved
    cyc = {"fused": [], "unfused": []}
    for _ in range(a.cycles):
        for mode in ("fused", "unfused"):
            mg.fused_restrict = mode == "fused"
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mg.cycle(bf)
            e1.record()
            e1.synchronize()
            cyc[mode].append(round(e0.elapsed_time(e1), 3))
    out["cycle_ms"] = cyc
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

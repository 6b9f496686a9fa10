#!/usr/bin/env python3
"""Where the v5 march spends its time: the clock-stamped diagnostic build (variant 114).

Runs the 515^3 p = 3 apply (and the Jacobi sweep) a few times with variant 114 and
reads the per-wave stamps (poms_diag_v5_stamps): cycles waiting for the wave's own
DMAs, in the plane barrier, and the rest (DMA issue, arithmetic, store); each wave's
start / end on the 100 MHz clock, its XCC and CU.  Prints the split, the spread of
workgroup durations, the per-CU busy time against the launch span, and the tail.

    python tools/v5_stamps.py --cells 512 --kinds apply,jacobi
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=512)
    ap.add_argument("--kinds", default="apply,jacobi")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default="")
    ap.add_argument("--chunk", type=int, default=0, help="axis-0 chunk (0: auto)")
    ap.add_argument("--per-tile", action="store_true", help="mean workgroup duration per tile row / column / chunk")
    ap.add_argument("--raw", default="", help="save per-workgroup start/end/XCD/CU of each rep to this .npz")
    ap.add_argument("--stamp-variant", type=int, default=114,
                    help="114: the production march stamped; 116: the software-pipelined apply stamped")
    a = ap.parse_args()
    import numpy as np
    import torch
    from poms_amd import _lib
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace

    p, N = 3, a.cells
    M, K = assemble_1d(uniform_knots(p, N), p)
    n = N + p
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    if a.chunk:
        A.set_chunk(a.chunk)
    x, b, y = V.zeros(), V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    out, raws = {}, {}
    for kind in a.kinds.split(","):
        fn = {"apply": lambda: A.dot(x, out=y),
              "jacobi": lambda: A.jacobi_sweep(b, x, y, 2.0 / 3.0, want_norm=False),
              "from_zero": lambda: A.jacobi_from_zero(b, y, 2.0 / 3.0, want_norm=True)}[kind]
        A.set_variant(10)
        for _ in range(3):
            fn()
        A.set_variant(a.stamp_variant)
        res = []
        for r in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            assert A.last_variant == a.stamp_variant
            nw = 1 << 16
            buf = (C.c_uint64 * (nw * 8))()
            _lib.call("poms_diag_v5_stamps", C.cast(buf, C.c_void_p), nw * 8)
            s = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 8).astype(np.float64)
            s = s[s[:, 3] > 0]   # waves that ran
            wait, bar, rest, planes, t0, t1, xcc, cu = s.T
            tile = np.floor(xcc / 256.0)   # the workgroup's tile (default-order index), stamped above the XCD id
            xcc = xcc - 256.0 * tile
            tot = wait + bar + rest
            wall_us = e0.elapsed_time(e1) * 1e3
            # workgroups: 16 waves each, consecutive rows
            nwg = len(s) // 16
            wg_t0 = t0[: nwg * 16].reshape(nwg, 16).min(1)
            wg_t1 = t1[: nwg * 16].reshape(nwg, 16).max(1)
            span = (wg_t1.max() - wg_t0.min()) / 100.0   # us
            wg_dur = (wg_t1 - wg_t0) / 100.0
            cuid = (xcc * 1000 + cu)[: nwg * 16].reshape(nwg, 16)[:, 0]
            busy = {}
            for c, d in zip(cuid, wg_dur):
                busy[c] = busy.get(c, 0.0) + d
            busyv = np.array(list(busy.values()))
            row = {"kind": kind, "rep": r, "event_us": wall_us, "span_us": span, "waves": int(len(s)), "wgs": nwg,
                   "cus_used": len(busy), "frac_wait": float(wait.sum() / tot.sum()),
                   "frac_barrier": float(bar.sum() / tot.sum()), "frac_rest": float(rest.sum() / tot.sum()),
                   "cycles_per_plane": float(tot.sum() / planes.sum()),
                   "wait_per_plane": float(wait.sum() / planes.sum()), "bar_per_plane": float(bar.sum() / planes.sum()),
                   "rest_per_plane": float(rest.sum() / planes.sum()),
                   "clock_ghz": float(tot.sum() / ((t1 - t0).sum() / 100.0) / 1e3),
                   "wg_us_median": float(np.median(wg_dur)), "wg_us_min": float(wg_dur.min()), "wg_us_max": float(wg_dur.max()),
                   "cu_busy_us_median": float(np.median(busyv)), "cu_busy_us_max": float(busyv.max()),
                   "cu_busy_us_min": float(busyv.min()), "util": float(busyv.sum() / (len(busy) * span)),
                   "tail_us": float((wg_t1.max() - np.sort(wg_t1)[int(0.9 * nwg)]) / 100.0)}
            # per tile row / column / chunk: mean workgroup duration (the stamped tile
            # index: t2 fastest, then t1, chunk -- the default POMS_TILE_ORDER)
            if a.per_tile:
                T2n, T1n = -(-(n) // 112), -(-(n) // 16)
                bids = tile[: nwg * 16].reshape(nwg, 16)[:, 0].astype(np.int64)
                t2s, t1s, chs = bids % T2n, (bids // T2n) % T1n, bids // (T1n * T2n)
                row["by_t1"] = {int(t): round(float(wg_dur[t1s == t].mean()), 1) for t in np.unique(t1s)}
                row["by_t2"] = {int(t): round(float(wg_dur[t2s == t].mean()), 1) for t in np.unique(t2s)}
                row["by_ch"] = {int(t): round(float(wg_dur[chs == t].mean()), 1) for t in np.unique(chs)}
            if a.raw:
                cus = (xcc + 0)[: nwg * 16].reshape(nwg, 16)[:, 0], cu[: nwg * 16].reshape(nwg, 16)[:, 0]
                raws[f"{kind}_{r}"] = np.stack([wg_t0, wg_t1, cus[0], cus[1], tile[: nwg * 16].reshape(nwg, 16)[:, 0]])
                # per wave (workgroup x wave): cycles waiting for own DMAs, in the barrier, the rest
                raws[f"{kind}_{r}_waves"] = np.stack([wait[: nwg * 16].reshape(nwg, 16), bar[: nwg * 16].reshape(nwg, 16),
                                                      rest[: nwg * 16].reshape(nwg, 16)])
            res.append(row)
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
        out[kind] = res
    A.set_variant(8)
    if a.raw:
        np.savez(a.raw, **raws)
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

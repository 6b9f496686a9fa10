#!/usr/bin/env python3
"""Interleaved A/B of the V-cycle under environment settings read per call
(POMS_PCG_SPEC, POMS_PCG_GRAPH, POMS_HOST_PARTIALS, ...), in ONE process, so that
box-to-box noise (the 2D bench varied 3.8-6.2 ms between runs of the same tree)
does not decide the comparison.

    python tools/cycle_ab.py --ndim 2 --cells 1024 --modes "POMS_PCG_GRAPH=0;POMS_PCG_GRAPH=1"

Each block runs --steps cycles per mode (modes in turn, --reps blocks); prints one
JSON line: per mode the min / median ms per cycle over the blocks, and the first
mode's x as the reference every other mode's x must equal bitwise.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=2)
    ap.add_argument("--cells", type=int, default=1024)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--coarse", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", type=str, default="POMS_PCG_GRAPH=0;POMS_PCG_GRAPH=1")
    a = ap.parse_args()
    import torch
    from poms_amd.mg import TwoLevelVCycle
    modes = []
    for m in a.modes.split(";"):
        env = dict(kv.split("=", 1) for kv in m.split(",") if kv)
        modes.append((m, env))
    mg = TwoLevelVCycle(a.p, a.cells, a.coarse, ndim=a.ndim)
    bf = mg.rhs_ones()

    def run(env, steps):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                x, _, _ = mg.cycle(bf)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / steps * 1e3, x
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    for _, env in modes:   # warm-up (captures, allocator)
        run(env, 3)
    times = {m: [] for m, _ in modes}
    stats = {m: {} for m, _ in modes}
    ref = None
    same = {m: True for m, _ in modes}
    for _ in range(a.reps):
        for m, env in modes:
            s0 = mg.A.spec_stats
            ms, x = run(env, a.steps)
            times[m].append(ms)
            for k, v in mg.A.spec_stats.items():
                stats[m][k] = stats[m].get(k, 0) + v - s0[k]
            xs = x._data.clone()
            if ref is None:
                ref = xs
            same[m] = same[m] and bool(torch.equal(xs, ref))
            del x
    out = {"ndim": a.ndim, "cells": a.cells, "p": a.p, "steps": a.steps, "reps": a.reps,
           "modes": {m: {"min_ms": min(t), "median_ms": statistics.median(t), "bitwise_equal_first": same[m],
                         "spec_stats": stats[m]}
                     for m, t in times.items()}}
    print(json.dumps(out))
    if not all(same.values()):
        raise SystemExit("modes disagree")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Wall-time breakdown of one two-level V-cycle (each phase synchronised):
where a host-bound configuration (2D p=3 1024^2) spends its cycle."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=2)
    ap.add_argument("--cells", type=int, default=1024)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from poms_amd.mg import TwoLevelVCycle
    from poms_amd.solvers import damped_jacobi, pcg
    torch.cuda.set_device(0)
    mg = TwoLevelVCycle(a.p, a.cells, 8, ndim=a.ndim)
    bf = mg.rhs_ones()
    A = mg.A
    for _ in range(2):
        mg.cycle(bf)
    torch.cuda.synchronize()
    acc = {}

    def t(name, fn):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + (time.perf_counter() - t0) * 1e3 / a.reps
        return r

    tw = time.perf_counter()
    for _ in range(a.reps):
        xf, _ = t("pcg_pre", lambda: pcg(A, damped_jacobi, bf, tol=mg.tol, maxiter=mg.maxiter))
        rf = t("residual", lambda: A.residual(bf, xf))
        rc = t("restrict", lambda: mg.transfer.restrict(rf, out=mg.rc))
        xc = t("coarse", lambda: mg.coarse_solve(rc, mg.xc))
        t("prolong", lambda: mg.transfer.prolong_add(xc, xf))
        t("ghosts", lambda: xf.update_ghost_regions())
        t("pcg_post", lambda: pcg(A, damped_jacobi, bf, x0=xf, tol=mg.tol, maxiter=mg.maxiter))
    V = mg.space
    rpre = V.empty()
    for _ in range(a.reps):
        t("x_empty", lambda: V.empty())
        t("x_residual_out", lambda: A.residual(bf, xf, out=rpre))
        t("x_residual_new", lambda: A.residual(bf, xf))
    acc["sum_ms"] = sum(v for k, v in acc.items() if not k.startswith("x_"))
    acc["wall_ms"] = (time.perf_counter() - tw) * 1e3 / a.reps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        mg.cycle(bf)
    torch.cuda.synchronize()
    acc["cycle_unsynced_ms"] = (time.perf_counter() - t0) * 1e3 / a.reps
    import gc
    for label, off in (("gc_on", False), ("gc_off", True)):
        if off:
            gc.collect()
            gc.disable()
        per = []
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mg.cycle(bf)
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) * 1e3)
        gc.enable()
        per.sort()
        acc[f"{label}_min_ms"], acc[f"{label}_median_ms"], acc[f"{label}_max_ms"] = per[0], per[10], per[-1]
    # unsynced: host time of each cycle call (the GPU may still be running)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(20):
        t1 = time.perf_counter()
        mg.cycle(bf)
        host.append(round((time.perf_counter() - t1) * 1e3, 2))
    torch.cuda.synchronize()
    acc["unsynced20_total_ms"] = (time.perf_counter() - t0) * 1e3
    acc["unsynced_host_per_cycle"] = host
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in acc.items()}), flush=True)


if __name__ == "__main__":
    main()

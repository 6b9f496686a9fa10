#!/usr/bin/env python3
"""Benchmark: two-level B-spline multigrid V-cycle, 3D -Δu+u, p=3, 512^3 cells
(``--ndim 2``: BASELINE config 2, 2D p=3 on a 1024^2 grid).

Contract (see the repo's task statement): ``python bench.py --gpus N --steps K
--warmup W``; for N > 1 launched by ``torch.distributed.run`` with one rank per
GPU (RCCL).  One *step* is one V-cycle of `sources/mg_jac.py:84-119`
(pcg(maxiter=10, tol=1e-6) pre-smoothing with 10-sweep damped-Jacobi
preconditioning, residual, restriction, coarse solve, prolongation, post
pcg) on the global grid, slab-decomposed over N GPUs (strong scaling).  Rank 0
prints ONE JSON line.

Reported beside the headline ``value`` (V-cycle DOF/s, whole job):
* ``roofline`` -- the dominant kernel (the fused Kron-apply + damped-Jacobi
  sweep, 24 algorithmic B/DOF) timed per launch with HIP events on the launch
  stream inside the timed region, against 8 TB/s;
* ``kron_spmv`` -- the plain Kron mat-vec (16 B/DOF) timed in isolation;
* ``cpu_baseline`` -- the C/OpenMP restatement of the reference loop nests
  running the same V-cycle on the host (rank 0, N = 1), bounded sample.

With ``--ndim 2`` the grid is 2D (N > 1: a Cart block decomposition, torch
transport) and the isolated mat-vec is timed after a 512 MiB MALL flush per launch
(a 1027^2 vector is 8.4 MB: without the flush it would be served from the
256 MB MALL / L2, not HBM).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "V-cycle DOF/s + Kron-SpMV GB/s vs HBM roofline, 3D Poisson p=3"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KERNEL_NAMES = {10: "kron_v5_kernel", 9: "kron_v3_kernel(flat)", 7: "kron_v4_kernel", 4: "kron_v3_kernel"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed V-cycles (default 3 in 3D, 20 in 2D)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed V-cycles (default 1 in 3D, 5 in 2D)")
    ap.add_argument("--ndim", type=int, default=3, choices=(2, 3))
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--cells", type=int, default=None, help="cells per axis (default 512 in 3D, 1024 in 2D)")
    ap.add_argument("--flush-mall", type=int, default=None,
                    help="MiB written between the isolated mat-vec launches (default 512 in 2D and for 3D grids "
                         "of <= 256 cells per axis, whose vectors fit the 256 MB MALL; 0 for the 512^3 headline)")
    ap.add_argument("--coarse", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--timing-every", type=int, default=4,
                    help="HIP events around every n-th Jacobi launch of the timed cycles (roofline.achieved)")
    ap.add_argument("--kron-reps", type=int, default=50, help="timed isolated applies")
    ap.add_argument("--kron-warm", type=int, default=30,
                    help="untimed applies before them: the apply's launch time falls from ~700 to ~530 us over "
                         "its first ~30 back-to-back launches at 515^3 (profiles/r03/kb_launch_series.log)")
    ap.add_argument("--cpu-cells", type=int, default=160,
                    help="cells per axis of the CPU baseline's V-cycle sample (all nproc cores)")
    ap.add_argument("--cpu-cycles", type=int, default=2)
    ap.add_argument("--cpu-cells-1core", type=int, default=64,
                    help="cells per axis of the single-core V-cycle sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", type=str, default=str(ROOT / "profiles" / "r06" / "pmc_traffic" / "pmc_traffic_jacobi.json"),
                    help="tools/pmc_traffic.py summary of a separate rocprofv3 --pmc pass "
                         "(FETCH_SIZE x2 + WRITE_SIZE per launch) used for roofline.traffic; used only "
                         "when its recorded p and kernel variant are this run's")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 3 if a.ndim == 3 else 50
    if a.warmup is None:
        # 2D: a cycle takes ~3.5 ms, and 5 untimed cycles left the GPU's clocks / the
        # host's state short of steady: 3.96-5.84 ms per cycle measured after 5, 3.44-3.59
        # after 200, on one box (profiles/r04/wu/)
        a.warmup = 1 if a.ndim == 3 else 200
    if a.cells is None:
        a.cells = 512 if a.ndim == 3 else 1024
    if a.flush_mall is None:   # configs whose working set fits the MALL are flushed
        a.flush_mall = 512 if (a.ndim == 2 or a.cells <= 256) else 0
    if a.ndim == 2 and a.cpu_cells == 160:
        a.cpu_cells = a.cells         # the 2D bench size runs on the host in seconds
    if a.ndim == 2 and a.cpu_cells_1core == 64:
        a.cpu_cells_1core = 256
    return a


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    from poms_amd.dist import CartDistribution, SlabDistribution
    from poms_amd.mg import TwoLevelVCycle

    nd = args.ndim
    n = args.cells + args.p
    comm_note = None
    if world == 1:
        dd = None
    elif nd == 3:
        # N > 1: the library's RCCL communicator.  It has never run with peers on the
        # builder's 1-GPU boxes: if it cannot be created or fails its self-test (every
        # rank raises together, the test ends in a MIN all-reduce) the bench runs on the
        # torch.distributed transport instead and SAYS so in "comm" / "comm_note".
        try:
            dd = SlabDistribution.from_process_group(n)
        except Exception as e:   # noqa: BLE001 -- reported in the JSON line
            comm_note = f"native RCCL communicator unavailable ({e!r:.300}); torch.distributed transport"
            os.environ["POMS_NATIVE_COMM"] = "0"
            dd = SlabDistribution.from_process_group(n)
    else:
        dd = CartDistribution.from_process_group((n, n))
    transport = dd.transport if dd is not None else "none"
    parallelism = (f"slab{world}" if nd == 3 else "cart" + "x".join(map(str, dd.dims))) if dd is not None else "slab1"
    mg = TwoLevelVCycle(args.p, args.cells, args.coarse, ndim=nd, dist=dd, chunk=args.chunk)
    bf = mg.rhs_ones()
    A = mg.A
    local_dof = 1
    for v in mg.space.local_npts:
        local_dof *= v

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        mg.cycle(bf)
    barrier()
    # HIP events around every --timing-every-th (default 4th) Jacobi launch of the timed region (a host event record
    # costs a few us: a sample keeps the measured cycle unperturbed)
    A.timing(True, "jacobi", every=args.timing_every, reserve=64 * args.steps + 64)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x, ipre, ipos = mg.cycle(bf)
    barrier()
    dt = time.perf_counter() - t0
    sweep_total_s, n_sweeps, sweep_dofs = A.timing_read("jacobi")
    A.timing(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    sec_per_cycle = dt / args.steps

    # per-launch kernel durations inside the timed region (events on the launch stream);
    # one operator call is 1 launch, or 2 when the halo exchange overlaps the interior planes
    def per_call(entries, want, stat="mean"):
        calls = {}
        for kind, e0, e1, call in entries:
            if kind == want:
                calls[call] = calls.get(call, 0.0) + e0.elapsed_time(e1) * 1e-3
        v = sorted(calls.values())
        if not v:
            return 0.0, 0
        if stat == "median":
            m = len(v) // 2
            return (v[m] if len(v) % 2 else 0.5 * (v[m - 1] + v[m])), len(v)
        return sum(v) / len(v), len(v)

    jac_v, app_v = A.kernel_variant("jacobi"), A.kernel_variant("apply")
    # average launch of the Jacobi sweep kernel (24 algorithmic B per output DOF); on a
    # slab one sweep is two launches (interior planes, then both boundaries)
    sweep_s = sweep_total_s / n_sweeps if n_sweeps else 0.0
    bytes_sweep = 24.0 * sweep_dofs / n_sweeps if n_sweeps else 0.0
    achieved = 24.0 * sweep_dofs / sweep_total_s / 1e9 if sweep_total_s > 0 else 0.0

    # isolated Kron mat-vec (16 B/DOF), same operator
    xv = mg.space.zeros()
    mg.space.interior(xv._data).uniform_(-1.0, 1.0)   # ghosts stay zero
    xv._mark_written()
    xv.update_ghost_regions()
    yk = mg.space.empty()
    for _ in range(max(3, args.kron_warm)):
        A.dot(xv, out=yk)
    flush = torch.empty(args.flush_mall * (1 << 17), dtype=torch.float64, device="cuda") if args.flush_mall else None
    barrier()
    A.timer = []
    for i in range(args.kron_reps):
        if flush is not None:
            flush.fill_(float(i))   # evict x, y and the factors from L2 / MALL (not timed)
        A.dot(xv, out=yk)
    barrier()
    del flush
    # the isolated apply: median over the launches (robust to the first launches after
    # the V-cycle, which run slower); the mean is reported beside it
    kron_s, _ = per_call(A.timer, "apply", "median")
    kron_mean_s, _ = per_call(A.timer, "apply")
    A.timer = None
    kron_gbps = 16.0 * local_dof / kron_s / 1e9 if kron_s > 0 else 0.0
    if world > 1:
        t = torch.tensor([achieved, kron_gbps], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        achieved, kron_gbps = (float(v) for v in t.tolist())

    traffic = None
    if args.pmc_json and Path(args.pmc_json).exists():
        pm = json.loads(Path(args.pmc_json).read_text())
        # per-DOF HBM bytes of the SAME kernel (order p, variant) scaled to this rank's slab
        if pm.get("bytes_per_dof") and pm.get("p") == args.p and pm.get("variant") == jac_v and \
                pm.get("ndim", 3) == nd:
            traffic = pm["bytes_per_dof"] * local_dof

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from oracle import cpu_baseline as cb
            host = cb.host_info()
            threads = host["nproc"]   # every CPU this process may use (GNU nproc)
            r = cb.time_vcycle(N=args.cpu_cells, p=args.p, Nc=args.coarse, cycles=args.cpu_cycles, threads=threads,
                               ndim=nd)
            r1 = cb.time_vcycle(N=args.cpu_cells_1core, p=args.p, Nc=args.coarse, cycles=1, threads=1, ndim=nd)
            full = cb.time_apply(N=args.cells, p=args.p, threads=threads, reps=2, ndim=nd)
            cpu = {"value": r["dof_per_s"], "unit": "DOF/s", "cores": r["threads"], "kind": "port",
                   "nproc": host["nproc"], "os_cpu_count": host["os_cpu_count"], "cpu_model": host["cpu_model"],
                   "sample": (f"{args.cpu_cycles} full two-level V-cycles (same schedule, incl. the reference's "
                              f"discarded mat-vec) at {args.cpu_cells}^{nd} cells p={args.p} ({r['dof']} DOF) on "
                              f"{r['threads']} threads, C/OpenMP restatement of the reference loop nests "
                              f"(oracle/kron_cpu.c), {r['seconds_per_cycle']:.2f} s per cycle; a bench-size "
                              f"({args.cells}^{nd}) CPU V-cycle is ~{r['seconds_per_cycle'] * (args.cells + args.p) ** nd / r['dof']:.1f} s "
                              f"at this rate" + (", outside the bounded sample" if args.cpu_cells != args.cells else "")),
                   "single_core": {"value": r1["dof_per_s"], "unit": "DOF/s", "cores": 1,
                                   "sample": f"1 V-cycle at {args.cpu_cells_1core}^{nd} cells ({r1['dof']} DOF), "
                                             f"{r1['seconds_per_cycle']:.2f} s"},
                   "kron_apply_full_size": {"value": full["gbps"], "unit": "GB/s (16 B/DOF)",
                                            "cores": full["threads"], "seconds_per_apply": full["seconds_per_apply"],
                                            "sample": f"{args.cells}^{nd} cells ({full['dof']} DOF), the bench size"}}
        except Exception as e:  # baseline is informative only
            cpu = {"value": None, "unit": "DOF/s", "cores": 0, "kind": "port", "sample": f"failed: {e!r}"}

    if rank == 0:
        gdof = mg.ndof
        out = {
            # BASELINE's metric names the headline 3D p = 3 config; other configs say theirs
            "metric": METRIC.replace("3D Poisson p=3", f"{nd}D Poisson p={args.p}"),
            "value": gdof / sec_per_cycle,
            "unit": "DOF/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": sec_per_cycle * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: b = 1 RHS (sources/mg_jac.py:57-62), uniform open knots, assembled -Δu+u factors",
            "config": {
                "workload": (f"two-level V-cycle, {nd}D -Δu+u, p={args.p}, {args.cells}^{nd} cells ({n}^{nd} DOF), "
                             f"coarse {args.coarse}^{nd} cells, pre/post pcg(tol=1e-6, maxiter=10) + damped Jacobi; "
                             f"the reference's discarded mat-vec s = A.dot(r) (sources/solvers.py:109, one per pcg "
                             f"iteration) is not computed on the GPU (the CPU baseline keeps it)"),
                "global_dof": gdof, "ndim": nd, "p": args.p, "cells": args.cells, "coarse_cells": args.coarse,
                "parallelism": parallelism,
            },
            "comm": transport,
            **({"comm_note": comm_note} if comm_note else {}),
            "roofline": {
                "kernel": f"{KERNEL_NAMES.get(jac_v, f'variant {jac_v}')}<P={args.p},{nd}D,SUM,JACOBI> (Kron apply + damped-Jacobi update)",
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                "algorithmic_bytes_per_launch": bytes_sweep, "avg_launch_us": sweep_s * 1e6,
                "launches_timed": n_sweeps,
            },
            "kron_spmv": {"kernel": f"{KERNEL_NAMES.get(app_v, f'variant {app_v}')}<P={args.p},{nd}D,SUM,APPLY>",
                          "mall_flush_mib": args.flush_mall,
                          "achieved": kron_gbps, "unit": "GB/s", "frac": kron_gbps / HBM_PEAK_GBPS,
                          "median_launch_us": kron_s * 1e6, "mean_launch_us": kron_mean_s * 1e6,
                          "bytes_per_dof": 16, "launches": args.kron_reps, "untimed_warmup_launches": args.kron_warm},
            "cpu_baseline": cpu,
            "solver": {"info_pre": ipre, "info_pos": ipos},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

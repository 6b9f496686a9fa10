"""One rank of the multi-process tests in tests/test_dist.py (launched as a subprocess
per rank with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment).

mode "cpu": gloo on CPU tensors -- slab split, p-plane ghost exchange, and a
slab-local Kronecker apply using the exchanged ghosts that must equal the
global oracle apply restricted to the slab (the decomposition is exact), plus
the restriction partial-sum + allreduce.

mode "gpu": gloo (host-staged exchange) with every rank on cuda:0 -- the
distributed KronOperator / vector algebra / transfer / two-level V-cycle of
poms_amd against the global single-process oracle.
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import poms_oracle as orc  # noqa: E402
from poms_amd.dist import SlabDistribution, slab_bounds  # noqa: E402
from poms_amd.splines import assemble_1d, band_to_dense, uniform_knots  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300))


def check(cond, msg):
    if not cond:
        raise AssertionError(f"rank {dist.get_rank()}: {msg}")


def slab_apply_local(ext, M, K, start, end, p):
    """Apply c M⊗M⊗M + K⊗M⊗M + M⊗K⊗M + M⊗M⊗K to the owned planes of a slab.

    ``ext`` holds planes [start - p, end + p) of x (ghosts from the neighbours,
    zeros past the global boundary); the axis-0 factor rows [start, end) see
    exactly those planes.
    """
    n0 = M.shape[0]
    Md, Kd = band_to_dense(M), band_to_dense(K)
    cols = np.arange(start - p, end + p)
    valid = (cols >= 0) & (cols < n0)

    def axis0(F):
        G = np.zeros((end - start, len(cols)))
        G[:, valid] = F[start:end][:, cols[valid]]
        return G

    def ap(F, X, axis):
        return np.moveaxis(np.tensordot(F, X, axes=([1], [axis])), 0, axis)

    M0, K0 = axis0(Md), axis0(Kd)
    mm = ap(Md, ap(Md, ext, 2), 1)
    y = ap(M0 + K0, mm, 0)
    y += ap(M0, ap(Kd, ap(Md, ext, 2), 1), 0)
    y += ap(M0, ap(Md, ap(Kd, ext, 2), 1), 0)
    return y


def run_cpu():
    rank, world = dist.get_rank(), dist.get_world_size()
    p, N = 3, 10
    n = N + p
    M, K = assemble_1d(uniform_knots(p, N), p)
    rng = np.random.default_rng(7)
    xg = rng.standard_normal((n, n, n))
    d = SlabDistribution.from_process_group(n)
    check((d.start, d.end) == slab_bounds(n, world, rank), "slab bounds")
    sizes = [slab_bounds(n, world, r)[1] - slab_bounds(n, world, r)[0] for r in range(world)]
    check(sum(sizes) == n and max(sizes) - min(sizes) <= 1, "split covers the axis evenly")
    # padded local slab (pads p on every axis), ghosts start as NaN sentinels
    loc = torch.full((d.n_local + 2 * p, n + 2 * p, n + 2 * p), float("nan"), dtype=torch.float64)
    loc[:, :p] = 0
    loc[:, -p:] = 0
    loc[:, :, :p] = 0
    loc[:, :, -p:] = 0
    loc[p:p + d.n_local, p:p + n, p:p + n] = torch.from_numpy(xg[d.start:d.end])
    if d.prev is None:
        loc[:p] = 0
    if d.next is None:
        loc[-p:] = 0
    h = d.start_exchange(loc, width=p, pad=p)
    d.finish_exchange(h)
    arr = loc.numpy()
    check(not np.isnan(arr).any(), "every ghost plane received")
    ext = arr[:, p:p + n, p:p + n]
    lo, hi = d.start - p, d.end + p
    want = np.zeros((hi - lo, n, n))
    a, b = max(lo, 0), min(hi, n)
    want[a - lo:b - lo] = xg[a:b]
    check(np.array_equal(ext, want), "ghost planes equal the neighbours' owned planes")
    y_loc = slab_apply_local(ext, M, K, d.start, d.end, p)
    y_glob = orc.kron_sum_apply(xg, [M] * 3, [K] * 3)[d.start:d.end]
    check(rel(y_loc, y_glob) <= 1e-14, f"slab apply {rel(y_loc, y_glob)}")
    # restriction: per-slab partial sums + allreduce == global restriction
    from poms_amd.splines import matrix_multi_stages
    from poms_amd.multilevels import knots_to_insert
    Tc, Tf = uniform_knots(p, 5), uniform_knots(p, N)
    ts = knots_to_insert(Tf, n, p, Tc, 5 + p, p)
    P1 = matrix_multi_stages(ts, 5 + p, p, Tc)
    part = np.einsum("ia,jb,kc,ijk->abc", P1[d.start:d.end], P1, P1, xg[d.start:d.end])
    t = torch.from_numpy(np.ascontiguousarray(part))
    from poms_amd.runtime import Comm
    comm = Comm.from_env()
    check(comm.enabled and comm.size == world and comm.rank == rank, "Comm from env")
    comm.allreduce_sum_(t)
    full = np.einsum("ia,jb,kc,ijk->abc", P1, P1, P1, xg)
    check(rel(t.numpy(), full) <= 1e-14, "restriction allreduce")
    check(abs(comm.allreduce_scalar(float(rank + 1)) - world * (world + 1) / 2) < 1e-12, "scalar allreduce")


def run_gpu():
    from poms_amd.mg import TwoLevelVCycle
    from poms_amd.multilevels import KronTransfer
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    p, N = 3, 14
    n = N + p
    M, K = assemble_1d(uniform_knots(p, N), p)
    rng = np.random.default_rng(3)
    xg, bg = rng.standard_normal((n, n, n)), rng.standard_normal((n, n, n))
    host_tr = os.environ.get("POMS_TEST_HOST_TRANSPORT") == "1"
    d = SlabDistribution.from_process_group(n, host_transport=host_tr)
    check(d.transport == ("native-host" if host_tr else "torch"), f"transport {d.transport}")
    V = StencilVectorSpace([n] * 3, [p] * 3, dist=d)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    sl = slice(d.start, d.end)
    Ag = orc.kron_sum_apply(xg, [M] * 3, [K] * 3)
    y = A.dot(x).to_local_numpy()
    check(rel(y, Ag[sl]) <= 1e-14, f"distributed apply {rel(y, Ag[sl])}")
    r = A.residual(b, x)
    check(rel(r.to_local_numpy(), (bg - Ag)[sl]) <= 1e-14, "distributed residual")
    D = orc.kron_sum_diag([M] * 3, [K] * 3).reshape(n, n, n)
    xo = V.zeros()
    nrm = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
    dr = 2.0 / 3.0 * (bg - Ag) / D
    check(rel(xo.to_local_numpy(), (xg + dr)[sl]) <= 1e-14, "distributed jacobi sweep")
    check(abs(nrm - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr)), "global sweep norm")
    if host_tr:   # the lazily read, all-reduced sweep norm through the C ring slots
        lz = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True, lazy=True)
        check(abs(lz.value() - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr)), "lazy global norm")
    g = x.dot(b)
    check(abs(g - float(np.vdot(xg, bg))) <= 1e-12 * abs(float(np.vdot(xg, bg))) + 1e-12, "global dot")
    # transfer: slab restriction + allreduce, prolongation on the owned planes
    from poms_amd.mg import two_level_setup_1d
    Tc, Tf = uniform_knots(p, 7), uniform_knots(p, N)
    _, _, P1 = two_level_setup_1d(p, Tf, Tc)
    tr = KronTransfer(V, [P1] * 3)
    rc = tr.restrict(x).cpu().numpy()
    full = np.einsum("ia,jb,kc,ijk->abc", P1, P1, P1, xg).reshape(-1)
    check(rel(rc, full) <= 1e-14, "distributed restriction")
    xc = rng.standard_normal(P1.shape[1] ** 3)
    z = V.zeros()
    tr.prolong_add(torch.from_numpy(xc).cuda(), z)
    pz = np.einsum("ia,jb,kc,abc->ijk", P1, P1, P1, xc.reshape((P1.shape[1],) * 3))
    check(rel(z.to_local_numpy(), pz[sl]) <= 1e-14, "distributed prolongation")
    # two-level V-cycle over the slabs vs the global oracle (p=2: stable smoother)
    devred = os.environ.get("POMS_TEST_DEVRED") == "1"
    mg = TwoLevelVCycle(2, 16, 4, ndim=3, dist=SlabDistribution.from_process_group(18, device_reductions=devred,
                                                                                   host_transport=host_tr))
    assert mg.space.lazy_reductions == devred or not devred
    bf = mg.rhs_ones()
    xf2, ipre, ipos = mg.cycle(bf)
    got = torch.from_numpy(xf2.toarray())
    dist.all_reduce(got)
    Mf, Kf = mg.M1d, mg.K1d
    ones = np.ones((mg.n,) * 3)
    xr, ipre_r, ipos_r = orc.vcycle_two_level([Mf] * 3, [Kf] * 3, mg.P1, ones)
    xr2, _, _ = orc.vcycle_two_level([Mf] * 3, [Kf] * 3, mg.P1, ones, reorder=True)
    tol = max(1e-9, 20 * rel(xr2, xr))
    err = rel(got.numpy().reshape(xr.shape), xr)
    check(err <= tol, f"distributed V-cycle {err} > {tol}")
    check(ipre["niter"] == ipre_r["niter"] and ipos["niter"] == ipos_r["niter"], "iteration counts")


def run_gpu_ksolve():
    """Distributed Kronecker direct solve: axis 0 by all-to-all transpose (gloo,
    host-staged) against the single-process oracle; 3 ranks make uneven splits."""
    from poms_amd.kron_solve import KronSolver
    from poms_amd.stencil import StencilVectorSpace
    torch.cuda.set_device(0)
    rng = np.random.default_rng(11)
    n, p = (13, 11, 9), 2
    F = []
    for d, (m, kl, ku) in enumerate(zip(n, (2, 1, 3), (1, 3, 2))):
        F.append(np.triu(np.tril(rng.uniform(-1, 1, (m, m)), ku), -kl) + 0.5 * np.eye(m))
    yg = rng.standard_normal(n)
    d = SlabDistribution.from_process_group(n[0])
    V = StencilVectorSpace(list(n), [p] * 3, dist=d)
    ks = KronSolver(V, F)
    y = V.zeros().from_numpy(yg)
    x = ks.solve(y).to_local_numpy()
    xg = orc.kron_solve(F, yg)
    check(rel(x, xg[d.start:d.end]) <= 1e-12, f"distributed kron solve {rel(x, xg[d.start:d.end])}")
    ks.solve(y, out=y)        # in place
    check(rel(y.to_local_numpy(), xg[d.start:d.end]) <= 1e-12, "distributed kron solve in place")


def main():
    mode = sys.argv[1]
    dist.init_process_group("gloo")
    try:
        {"cpu": run_cpu, "gpu": run_gpu, "gpu_ksolve": run_gpu_ksolve}[mode]()
        dist.barrier()
        print(f"rank {dist.get_rank()} ok", flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

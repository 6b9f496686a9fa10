"""One rank of the multi-process tests in tests/test_dist.py (launched as a subprocess
per rank with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment).

mode "cpu": gloo on CPU tensors -- slab split, p-plane ghost exchange, and a
slab-local Kronecker apply using the exchanged ghosts that must equal the
global oracle apply restricted to the slab (the decomposition is exact), plus
the restriction partial-sum + allreduce.

mode "cart_cpu" / "cart_gpu": the same over a Cart block decomposition of every
axis (POMS_TEST_CART_DIMS, e.g. "2x2x1"), 4 ranks.

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
    host_shm = os.environ.get("POMS_TEST_HOST_SHM") == "1"
    d = SlabDistribution.from_process_group(n, host_transport=host_tr, host_shm=host_shm)
    world = dist.get_world_size()
    check(d.transport == ("none" if world == 1 else "native-host" if host_tr else "torch"), f"transport {d.transport}")
    if host_tr:   # the host-read sums take the node-local shared-memory block when asked
        check(d.native.uses_shm == host_shm, f"shm attached {d.native.uses_shm}")
    V = StencilVectorSpace([n] * 3, [p] * 3, dist=d)
    A = KronOperator.laplace(V, [M] * 3, [K] * 3)
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    if world == 1 and host_tr:
        # one rank, no neighbour: poms_op_run_dist itself (the space is not distributed, so
        # only a direct call reaches it) must take the single-launch path -- no exchange is
        # queued -- and equal the plain launch bitwise, sums included
        y_ref, xo_ref = A.dot(x), V.zeros()
        nrm_ref = A.jacobi_sweep(b, x, xo_ref, 2.0 / 3.0, want_norm=True)
        for _ in range(3):
            x._ghost_valid = False   # asks for an exchange, which has no neighbour to go to
            y = V.zeros()
            A._run_native("apply", x, y)
            check(bool(torch.equal(y._data, y_ref._data)), "no-neighbour run_dist apply")
            x._ghost_valid = False
            xo, nd = V.zeros(), torch.zeros(1, dtype=torch.float64, device="cuda")
            A._run_native("jacobi", x, xo, b, omega=2.0 / 3.0, norm_out=nd)
            check(bool(torch.equal(xo._data, xo_ref._data)), "no-neighbour run_dist jacobi")
            check(abs(float(nd) - nrm_ref) <= 1e-13 * nrm_ref, f"no-neighbour run_dist norm {float(nd)} vs {nrm_ref}")
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
    # fused residual -> restriction over the slabs (no ghost planes needed) + allreduce
    x._ghost_valid = False
    rcf = tr.resid_restrict(A, b, x).cpu().numpy()
    fullr = np.einsum("ia,jb,kc,ijk->abc", P1, P1, P1, bg - Ag).reshape(-1)
    check(rel(rcf, fullr) <= 1e-13, f"distributed fused residual -> restriction {rel(rcf, fullr)}")
    # two-level V-cycle over the slabs vs the global oracle (p=2: stable smoother)
    devred = os.environ.get("POMS_TEST_DEVRED") == "1"
    mg = TwoLevelVCycle(2, 16, 4, ndim=3, dist=SlabDistribution.from_process_group(18, device_reductions=devred,
                                                                                   host_transport=host_tr,
                                                                                   host_shm=host_shm))
    assert mg.space.lazy_reductions == devred or not devred
    check(mg.fused_restrict, "the V-cycle takes the fused residual -> restriction")
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
    _check_peer(d)
    _check_peer(mg.space.dist)


def _check_peer(d):
    """With POMS_COMM_PEER=1 every exchange went through the peer transport, and no
    wait of its kernel timed out."""
    want = os.environ.get("POMS_COMM_PEER") == "1"
    nc = getattr(d, "native", None)
    if nc is None or dist.get_world_size() == 1:
        return
    check(nc.peer == want, f"peer transport {nc.peer}, asked {want}")
    if want:
        st = nc.peer_status()
        check(st["active"] and not st["timed_out"], f"peer transport status {st}")


def run_gpu_fullsize_slabs():
    """The headline grid (515^3, p = 3; POMS_TEST_FULL_N cells) split over the ranks
    exactly as the 8-GPU run splits it (65/64-plane slabs), every rank on cuda:0, the
    production schedule (poms_op_run_dist, poms_pcg_jacobi) over the host transport
    with the node-local shared-memory sums attached -- the code the driver's 8-GPU run
    executes, bar RCCL's byte moves.  Each rank also builds the whole grid and runs
    the same operations on one GPU; its slab of every result must agree to 1e-13
    (fixed counts: apply, residual, a Jacobi sweep and its norm, the lazily read norm,
    damped Jacobi, pcg with damped Jacobi) with identical iteration counts
    (`sources/solvers.py:69-135, 167-235`)."""
    import torch
    from poms_amd import solvers
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    p, N = 3, int(os.environ.get("POMS_TEST_FULL_N", "512"))
    n = N + p
    M, K = assemble_1d(uniform_knots(p, N), p)
    d = SlabDistribution.from_process_group(n, host_transport=True, host_shm=True)
    check(d.native.uses_shm, "node-local shared-memory sums attached")
    Vl = StencilVectorSpace([n] * 3, [p] * 3, dist=d, align=True)
    Al = KronOperator.laplace(Vl, [M] * 3, [K] * 3)
    Vg = StencilVectorSpace([n] * 3, [p] * 3, align=True)
    Ag = KronOperator.laplace(Vg, [M] * 3, [K] * 3)
    gen = torch.Generator(device="cuda").manual_seed(17)
    xg, bg = Vg.zeros(), Vg.zeros()
    Vg.interior(xg._data).uniform_(-1, 1, generator=gen)
    Vg.interior(bg._data).uniform_(-1, 1, generator=gen)
    sl = slice(d.start, d.end)

    def local(vg):
        v = Vl.zeros()
        Vl.interior(v._data).copy_(Vg.interior(vg._data)[sl])
        v._mark_written()   # the ghosts now stale: the next operator call exchanges them
        return v

    def cmp(tag, vl, vg, tol=1e-13):
        a, b = Vl.interior(vl._data), Vg.interior(vg._data)[sl]
        err = float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))
        check(err <= tol, f"{tag}: slab vs one GPU, rel {err:.3e}")
        return err

    xl, bl = local(xg), local(bg)
    errs = {"apply": cmp("apply", Al.dot(xl), Ag.dot(xg))}
    errs["residual"] = cmp("residual", Al.residual(bl, xl), Ag.residual(bg, xg))
    w = 2.0 / 3.0
    xol, xog = Vl.zeros(), Vg.zeros()
    nl = Al.jacobi_sweep(bl, xl, xol, w, want_norm=True)
    ng = Ag.jacobi_sweep(bg, xg, xog, w, want_norm=True)
    errs["jacobi"] = cmp("jacobi sweep", xol, xog)
    check(abs(nl - ng) <= 1e-13 * ng, f"sweep norm {nl} vs {ng}")
    lz = Al.jacobi_sweep(bl, xl, xol, w, want_norm=True, lazy=True)
    check(abs(lz.value() - ng) <= 1e-13 * ng, f"lazy (shared-memory) sweep norm {lz.value()} vs {ng}")
    errs["damped_jacobi"] = cmp("damped_jacobi", solvers.damped_jacobi(Al, bl, maxiter=10),
                                solvers.damped_jacobi(Ag, bg, maxiter=10))
    for m in (1, 2):
        xl2, il = solvers.pcg(Al, solvers.damped_jacobi, bl, tol=0.0, maxiter=m)
        xg2, ig = solvers.pcg(Ag, solvers.damped_jacobi, bg, tol=0.0, maxiter=m)
        check(il["niter"] == ig["niter"] == m, f"pcg niter {il['niter']} / {ig['niter']}")
        errs[f"pcg{m}"] = cmp(f"pcg maxiter {m}", xl2, xg2)
        check(abs(il["res_norm"] - ig["res_norm"]) <= 1e-12 * ig["res_norm"], f"pcg res_norm {il} {ig}")
    # the reference's stop test decides (tol 1e-6): both stop at the same iteration
    xl3, il = solvers.pcg(Al, solvers.damped_jacobi, bl, tol=1e-6, maxiter=10)
    xg3, ig = solvers.pcg(Ag, solvers.damped_jacobi, bg, tol=1e-6, maxiter=10)
    check(il["niter"] == ig["niter"] and il["success"] == ig["success"], f"pcg stop {il} vs {ig}")
    _check_peer(d)
    print(f"rank {dist.get_rank()} slab [{d.start}, {d.end}) errors {errs}", flush=True)


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


def _cart_dims():
    return tuple(int(v) for v in os.environ["POMS_TEST_CART_DIMS"].split("x"))


def block_apply_local(ext, Ms, Ks, starts, ends, p, c=1.0):
    """c M⊗M(⊗M) + the stiffness terms applied to the owned block of a Cart rank.

    ``ext`` holds x on the window ``[starts[d] - p, ends[d] + p)`` of every axis
    (ghosts from the neighbours, zeros past the global boundary); factor rows are
    the owned rows, columns that window."""
    nd = len(starts)

    def loc(F, d):
        n = F.shape[0]
        Fd = band_to_dense(F)
        cols = np.arange(starts[d] - p, ends[d] + p)
        valid = (cols >= 0) & (cols < n)
        G = np.zeros((ends[d] - starts[d], len(cols)))
        G[:, valid] = Fd[starts[d]:ends[d]][:, cols[valid]]
        return G

    def ap(F, X, axis):
        return np.moveaxis(np.tensordot(F, X, axes=([1], [axis])), 0, axis)

    Ml = [loc(M, d) for d, M in enumerate(Ms)]
    Kl = [loc(K, d) for d, K in enumerate(Ks)]
    y = ext
    for d in range(nd):
        y = ap(Ml[d], y, d)
    y = c * y
    for k in range(nd):
        t = ext
        for d in range(nd):
            t = ap(Kl[d] if d == k else Ml[d], t, d)
        y = y + t
    return y


def run_cart_cpu():
    """Cart block decomposition on CPU tensors: the ghost layers of every decomposed
    axis (edges and corners included) equal the neighbours' owned entries, and a
    block-local apply on them equals the global oracle's rows."""
    from poms_amd.dist import CartDistribution
    rank, world = dist.get_rank(), dist.get_world_size()
    dims = _cart_dims()
    nd = len(dims)
    p, N = 3, 9
    n = N + p
    M, K = assemble_1d(uniform_knots(p, N), p)
    rng = np.random.default_rng(5)
    xg = rng.standard_normal((n,) * nd)
    d = CartDistribution.from_process_group((n,) * nd, dims)
    check(d.dims == dims and d.world == world and d.rank_of(d.coords) == rank, "grid")
    for ax in range(nd):
        b = [slab_bounds(n, dims[ax], c) for c in range(dims[ax])]
        check((d.starts[ax], d.ends[ax]) == b[d.coords[ax]], f"axis {ax} bounds")
    # every owned point exactly once over the ranks
    own = torch.zeros((n,) * nd, dtype=torch.float64)
    own[tuple(slice(s, e) for s, e in zip(d.starts, d.ends))] = 1.0
    dist.all_reduce(own)
    check(bool((own == 1.0).all()), "blocks tile the grid")
    shape = tuple(nl + 2 * p for nl in d.n_local)
    loc = torch.full(shape, float("nan"), dtype=torch.float64)
    inner = tuple(slice(p, p + nl) for nl in d.n_local)
    loc[inner] = torch.from_numpy(xg[tuple(slice(s, e) for s, e in zip(d.starts, d.ends))])
    # ghosts past the global boundary are zero; the rest come from the exchange
    for ax in range(nd):
        for side, nbr in ((0, d.prev[ax]), (1, d.next[ax])):
            if nbr is None:
                idx = [slice(None)] * nd
                idx[ax] = slice(0, p) if side == 0 else slice(p + d.n_local[ax], None)
                loc[tuple(idx)] = 0.0
    d.exchange(loc, (p,) * nd)
    arr = loc.numpy()
    check(not np.isnan(arr).any(), "every ghost (edges, corners) received")
    want = np.zeros(shape)
    src = tuple(slice(max(s - p, 0), min(e + p, n)) for s, e in zip(d.starts, d.ends))
    dst = tuple(slice(max(s - p, 0) - (s - p), min(e + p, n) - (s - p)) for s, e in zip(d.starts, d.ends))
    want[dst] = xg[src]
    check(np.array_equal(arr, want), "ghost layers equal the neighbours' owned entries")
    y = block_apply_local(arr, [M] * nd, [K] * nd, d.starts, d.ends, p)
    Ag = orc.kron_sum_apply(xg, [M] * nd, [K] * nd) if nd == 3 else None
    if Ag is None:
        Md, Kd = band_to_dense(M), band_to_dense(K)
        Ag = Md @ xg @ Md.T + Kd @ xg @ Md.T + Md @ xg @ Kd.T
    own_sl = tuple(slice(s, e) for s, e in zip(d.starts, d.ends))
    check(rel(y, Ag[own_sl]) <= 1e-14, f"block apply {rel(y, Ag[own_sl])}")


def _cart_ops(d, nd, p, N, align):
    """Operator, sweep, reductions and transfer on one Cart space vs the oracle."""
    from poms_amd.multilevels import KronTransfer
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    n = N + p
    tag = f"p={p} align={align}"
    M, K = assemble_1d(uniform_knots(p, N), p)
    rng = np.random.default_rng(3)
    xg, bg = rng.standard_normal((n,) * nd), rng.standard_normal((n,) * nd)
    V = StencilVectorSpace([n] * nd, [p] * nd, dist=d, align=align)
    check(V.is_cart and V.starts == d.starts, "space block")
    A = KronOperator.laplace(V, [M] * nd, [K] * nd)
    check(not A.from_zero_supported, "no from-zero sweeps on a Cart block")
    x, b = V.zeros().from_numpy(xg), V.zeros().from_numpy(bg)
    sl = tuple(slice(s, e) for s, e in zip(d.starts, d.ends))
    Md, Kd = band_to_dense(M), band_to_dense(K)
    if nd == 3:
        Ag = orc.kron_sum_apply(xg, [M] * 3, [K] * 3)
        D = orc.kron_sum_diag([M] * 3, [K] * 3).reshape((n,) * 3)
    else:
        Ag = Md @ xg @ Md.T + Kd @ xg @ Md.T + Md @ xg @ Kd.T
        dm, dk = np.diag(Md), np.diag(Kd)
        D = np.outer(dm, dm) + np.outer(dk, dm) + np.outer(dm, dk)
    y = A.dot(x).to_local_numpy()
    # the exchanged padded block equals the global window (zeros past the boundary)
    win = np.zeros(tuple(nl + 2 * p for nl in d.n_local))
    src = tuple(slice(max(s - p, 0), min(e + p, n)) for s, e in zip(d.starts, d.ends))
    dst = tuple(slice(max(s - p, 0) - (s - p), min(e + p, n) - (s - p)) for s, e in zip(d.starts, d.ends))
    win[dst] = xg[src]
    check(np.array_equal(x._data.cpu().numpy(), win), f"{tag}: device ghost layers")
    check(rel(y, Ag[sl]) <= 1e-14, f"{tag}: Cart apply {rel(y, Ag[sl])}")
    # every kernel variant reads the exchanged ghosts of the decomposed axes
    v0 = A.variant
    errs = {}
    for v in (0, 4, 7, 9, 10):
        A.set_variant(v)
        yv = A.dot(V.zeros().from_numpy(xg)).to_local_numpy()
        errs[(v, A.kernel_variant("apply"))] = rel(yv, Ag[sl])
        bad = np.argwhere(np.abs(yv - Ag[sl]) > 1e-12 * np.abs(Ag).max())
        if len(bad):
            print(f"rank {dist.get_rank()} {tag} variant {v}: {len(bad)} bad points, first {bad[:6].tolist()}",
                  flush=True)
    A.set_variant(v0)
    check(all(e <= 1e-14 for e in errs.values()), f"{tag}: Cart apply by variant {errs}")
    r = A.residual(b, x)
    check(rel(r.to_local_numpy(), (bg - Ag)[sl]) <= 1e-14, f"{tag}: Cart residual")
    xo = V.zeros()
    nrm = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
    dr = 2.0 / 3.0 * (bg - Ag) / D
    check(rel(xo.to_local_numpy(), (xg + dr)[sl]) <= 1e-14, f"{tag}: Cart jacobi sweep")
    check(abs(nrm - float(np.vdot(dr, dr))) <= 1e-12 * float(np.vdot(dr, dr)), f"{tag}: global sweep norm")
    z = V.zeros()
    nz = A.diag_scale(b, z, 2.0 / 3.0, want_norm=True)
    zr = 2.0 / 3.0 * bg / D
    check(rel(z.to_local_numpy(), zr[sl]) <= 1e-15, f"{tag}: Cart diag_scale {rel(z.to_local_numpy(), zr[sl])}")
    check(abs(nz - float(np.vdot(zr, zr))) <= 1e-12 * float(np.vdot(zr, zr)), f"{tag}: diag_scale norm")
    nrm2, dot2 = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True, want_dot=True)
    want = float(np.vdot(xg + dr, bg))
    check(abs(dot2 - want) <= 1e-12 * abs(want), f"{tag}: sweep + fused dot")
    pq = A.dot_inner(x, xo)
    want = float(np.vdot(xg, Ag))
    check(abs(pq - want) <= 1e-12 * abs(want), f"{tag}: Cart apply + fused dot")
    g = x.dot(b)
    check(abs(g - float(np.vdot(xg, bg))) <= 1e-12 * abs(float(np.vdot(xg, bg))) + 1e-12, f"{tag}: global dot")
    # spl-style single-axis ghost updates, then an apply on the already-valid ghosts
    x2 = V.zeros().from_numpy(xg)
    for ax in range(nd):
        x2.update_ghost_regions(direction=ax)
    x2._ghost_valid = True
    check(rel(A.dot(x2).to_local_numpy(), Ag[sl]) <= 1e-14, f"{tag}: apply after per-axis updates")
    # transfer: block restriction + allreduce, prolongation on the owned block
    from poms_amd.mg import two_level_setup_1d
    Tc, Tf = uniform_knots(p, N // 2), uniform_knots(p, N)
    _, _, P1 = two_level_setup_1d(p, Tf, Tc)
    tr = KronTransfer(V, [P1] * nd)
    rc = tr.restrict(x).cpu().numpy()
    if nd == 3:
        full = np.einsum("ia,jb,kc,ijk->abc", P1, P1, P1, xg).reshape(-1)
    else:
        full = (P1.T @ xg @ P1).reshape(-1)
    check(rel(rc, full) <= 1e-14, f"{tag}: Cart restriction")
    nc = P1.shape[1]
    xc = rng.standard_normal(nc ** nd)
    z = V.zeros()
    tr.prolong_add(torch.from_numpy(xc).cuda(), z)
    if nd == 3:
        pz = np.einsum("ia,jb,kc,abc->ijk", P1, P1, P1, xc.reshape((nc,) * 3))
    else:
        pz = P1 @ xc.reshape(nc, nc) @ P1.T
    check(rel(z.to_local_numpy(), pz[sl]) <= 1e-14, f"{tag}: Cart prolongation")
    # fused residual -> restriction on the block (G rows sliced like P's) + allreduce
    rcf = tr.resid_restrict(A, b, x).cpu().numpy()
    rg = bg - Ag
    fullr = (np.einsum("ia,jb,kc,ijk->abc", P1, P1, P1, rg) if nd == 3 else P1.T @ rg @ P1).reshape(-1)
    check(rel(rcf, fullr) <= 1e-13, f"{tag}: Cart fused residual -> restriction {rel(rcf, fullr)}")


def run_cart_gpu():
    """The device operator, vector algebra, transfer and two-level V-cycle over a
    Cart block decomposition (gloo, every rank on cuda:0) against the global oracle."""
    from poms_amd.dist import CartDistribution
    from poms_amd.mg import TwoLevelVCycle
    torch.cuda.set_device(0)
    dims = _cart_dims()
    nd = len(dims)
    for p, N, align in ((3, 14, False), (3, 14, True), (2, 16, True), (1, 10, False)):
        d = CartDistribution.from_process_group((N + p,) * nd, dims, device_reductions=True)
        check(d.transport == "torch", "transport")
        _cart_ops(d, nd, p, N, align)
    # two-level V-cycle (p=2) over the blocks vs the global oracle
    nf = 18
    errs = []
    for devred in (False, True):
        mg = TwoLevelVCycle(2, 16, 4, ndim=nd, dist=CartDistribution.from_process_group(
            (nf,) * nd, dims, device_reductions=devred))
        bf = mg.rhs_ones()
        xf2, ipre, ipos = mg.cycle(bf)
        got = torch.from_numpy(xf2.toarray())
        dist.all_reduce(got)
        ones = np.ones((mg.n,) * nd)
        xr, ipre_r, ipos_r = orc.vcycle_two_level([mg.M1d] * nd, [mg.K1d] * nd, mg.P1, ones)
        xr2, _, _ = orc.vcycle_two_level([mg.M1d] * nd, [mg.K1d] * nd, mg.P1, ones, reorder=True)
        tol = max(1e-9, 20 * rel(xr2, xr))
        err = rel(got.numpy().reshape(xr.shape), xr)
        errs.append((devred, err, tol, ipre["niter"], ipre_r["niter"], ipos["niter"], ipos_r["niter"]))
    # the same V-cycle on one rank (no decomposition) through the same code
    from poms_amd.stencil import StencilVectorSpace
    mg1 = TwoLevelVCycle(2, 16, 4, ndim=nd)
    x1, _, _ = mg1.cycle(mg1.rhs_ones())
    errs.append(("single", rel(x1.toarray().reshape(xr.shape), xr)))
    for e in errs[:2]:
        devred, err, tol = e[:3]
        check(err <= tol, f"Cart V-cycle (device reductions {devred}) {err} > {tol}; all {errs}")
        check(e[3] == e[4] and e[5] == e[6], f"iteration counts {errs}")


def run_cart_ksolve():
    """Kronecker direct solve over a Cart block decomposition (every split axis
    solved by line-group transposes, `sources/kron_product.py:119-170, 191-238`)
    against the single-process oracle, and pcg_glt (`sources/solvers.py:239-306`)
    over 2D blocks against the reference's golden iterates (tests/golden/pcg_glt.npz)."""
    from poms_amd.dist import CartDistribution
    from poms_amd.kron_solve import KronSolver
    from poms_amd.solvers import pcg_glt
    from poms_amd.splines import assemble_1d, make_open_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    dims = _cart_dims()
    nd = len(dims)
    rng = np.random.default_rng(29)
    n = (13, 11, 9)[3 - nd:] if nd == 3 else (13, 11)
    F = []
    for m, kl, ku in zip(n, (2, 1, 3), (1, 3, 2)):
        F.append(np.triu(np.tril(rng.uniform(-1, 1, (m, m)), ku), -kl) + 0.5 * np.eye(m))
    yg = rng.standard_normal(n)
    xg = orc.kron_solve(F, yg)
    for p, align in ((2, False), (3, True)):
        d = CartDistribution.from_process_group(n, dims)
        V = StencilVectorSpace(list(n), [p] * nd, dist=d, align=align)
        ks = KronSolver(V, F)
        sl = tuple(slice(s, e) for s, e in zip(d.starts, d.ends))
        y = V.zeros().from_numpy(yg)
        x = ks.solve(y).to_local_numpy()
        check(rel(x, xg[sl]) <= 1e-12, f"Cart kron solve p={p} {rel(x, xg[sl])}")
        ks.solve(y, out=y)   # in place
        check(rel(y.to_local_numpy(), xg[sl]) <= 1e-12, f"Cart kron solve in place p={p}")
    if nd != 2:
        return
    z = np.load(Path(__file__).with_name("golden") / "pcg_glt.npz", allow_pickle=False)
    cases = {}
    for k in z.files:
        case, field = k.split("__", 1)
        cases.setdefault(case, {})[field] = z[k]
    for name in ("p2_ne8", "p3_ne12"):
        c = cases[name]
        p, ne = int(c["p"]), int(c["ne"])
        M, K = assemble_1d(make_open_knots(p, ne + p), p)
        nn = ne + p
        d = CartDistribution.from_process_group((nn, nn), dims)
        V = StencilVectorSpace([nn, nn], [p, p], dist=d)
        A = KronOperator.laplace(V, [M, M], [K, K])
        b = V.zeros().from_numpy(c["b"].reshape(nn, nn))
        for m in (1, 3):   # fixed iteration counts: the reference's iterates at 1e-9
            x, info = pcg_glt(A, c["M1"], c["M2"], b, tol=0.0, maxiter=m)
            got = torch.from_numpy(x.toarray())
            dist.all_reduce(got)
            check(info["niter"] == int(c[f"glt_m{m}_tol0_info"][0]), f"{name} m={m} niter")
            check(rel(got.numpy(), c[f"glt_m{m}_tol0"]) <= 1e-9, f"{name} m={m}: {rel(got.numpy(), c[f'glt_m{m}_tol0'])}")
        x, info = pcg_glt(A, c["M1"], c["M2"], b, tol=1e-8, maxiter=100)
        check(info["niter"] == int(c["glt_test_info"][0]) and info["success"] == bool(c["glt_test_info"][1]),
              f"{name}: converged niter {info['niter']} vs {c['glt_test_info']}")


def main():
    mode = sys.argv[1]
    dist.init_process_group("gloo")
    try:
        {"cpu": run_cpu, "gpu": run_gpu, "gpu_ksolve": run_gpu_ksolve, "gpu_fullsize_slabs": run_gpu_fullsize_slabs,
         "cart_cpu": run_cart_cpu,
         "cart_gpu": run_cart_gpu, "cart_ksolve": run_cart_ksolve}[mode]()
        dist.barrier()
        print(f"rank {dist.get_rank()} ok", flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

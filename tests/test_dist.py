"""Multi-process slab decomposition (world_size 2, gloo): one subprocess per rank."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from poms_amd.dist import CartDistribution, dims_create, slab_bounds

WORKER = Path(__file__).with_name("dist_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(mode, world=2, timeout=300, extra_env=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, str(WORKER), mode], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    failed = [(r, rc, out) for r, (rc, out) in enumerate(outs) if rc != 0]
    if failed:
        # the rank whose own check failed first, not a peer that lost its connection
        failed.sort(key=lambda f: "AssertionError" not in f[2])
        r, rc, out = failed[0]
        others = [ln for _, _, o in failed[1:] for ln in o.splitlines() if "AssertionError" in ln]
        raise AssertionError(f"rank {r} failed (rc={rc}):\n{out[-4000:]}\nother ranks:\n" + "\n".join(others))
    for r, (rc, out) in enumerate(outs):
        assert f"rank {r} ok" in out


@pytest.mark.parametrize("n,w", [(515, 8), (515, 1), (17, 2), (16, 4), (10, 3)])
def test_slab_bounds(n, w):
    b = [slab_bounds(n, w, r) for r in range(w)]
    assert b[0][0] == 0 and b[-1][1] == n
    assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
    sizes = [e - s for s, e in b]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    if (n, w) == (515, 8):
        assert sizes == [65, 65, 65, 64, 64, 64, 64, 64]


def test_slab_distribution_rejects_thin_slabs():
    from poms_amd.dist import SlabDistribution
    with pytest.raises(ValueError):
        SlabDistribution(3, 3, 4)
    d = SlabDistribution(17, 1, 2)
    assert (d.start, d.end, d.prev, d.next) == (9, 17, 0, None)


def test_two_rank_halo_exchange_and_slab_apply_cpu():
    _launch("cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("device_reductions", [False, True])
def test_two_rank_distributed_operator_and_vcycle_gpu(device_reductions):
    """device_reductions: the global sums stay device tensors (gloo reduces CUDA
    tensors), which runs the RCCL configuration's device-scalar pcg path."""
    # device_count() does not initialise HIP in this (parent) process: the ranks
    # are the only processes that touch the GPU here
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    _launch("gpu", extra_env={"POMS_TEST_DEVRED": "1" if device_reductions else "0"})


@pytest.mark.gpu
@pytest.mark.parametrize("world,boundary_on_cs,shm,peer", [(2, "1", "0", "0"), (3, "1", "0", "0"), (2, "0", "0", "0"),
                                                           (2, "1", "1", "0"), (3, "1", "1", "0"), (1, "1", "0", "0"),
                                                           (2, "1", "1", "1"), (3, "1", "1", "1"), (3, "0", "1", "1")])
def test_two_rank_native_schedule_with_peers_gpu(world, boundary_on_cs, shm, peer):
    """The production slab schedule (poms_op_run_dist: exchange, interior planes,
    both boundaries in one launch -- on the communication stream behind the
    exchange, or with POMS_BOUNDARY_ON_CS=0 on the compute stream; lazy ring-slot
    norms; device-scalar pcg; restriction all-reduce through the library
    communicator) with REAL neighbours: the communicator's host transport moves the
    planes and sums over gloo, since RCCL cannot pair ranks that share one GPU.
    shm=1: the host-read sums go through the node-local shared-memory block
    (shm_allsum, poms_comm_wait's shared-memory branch) as in a one-node RCCL run.
    world=1: a communicator with no neighbour takes the single-launch path (no
    exchange is queued, so no split launch may run unordered on the communication
    stream; advisor, round 3).  peer=1: the ghost planes move through the peer
    transport instead (POMS_COMM_PEER: one kernel on the communication stream storing
    into the neighbours' IPC-mapped mailboxes -- here processes sharing the GPU)."""
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    _launch("gpu", world=world, extra_env={"POMS_TEST_DEVRED": "1", "POMS_TEST_HOST_TRANSPORT": "1",
                                           "POMS_BOUNDARY_ON_CS": boundary_on_cs, "POMS_TEST_HOST_SHM": shm,
                                           "POMS_COMM_PEER": peer})


@pytest.mark.gpu
@pytest.mark.parametrize("peer", ["0", "1"])
def test_eight_rank_fullsize_slabs_host_transport_gpu(peer):
    """The 8-GPU run's split of the headline grid (515^3 over 8 ranks: 65/64-plane
    slabs) on one GPU: the production schedule and the shared-memory sums against
    the single-GPU result at 1e-13 with identical iteration counts.  peer=1: the
    ghost exchange through the peer transport (POMS_COMM_PEER)."""
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    # (8 exchange workgroups per rank: each holds a CU slot while it waits for its
    # neighbours, and here 8 ranks share one GPU)
    _launch("gpu_fullsize_slabs", world=8, timeout=900, extra_env={"POMS_COMM_PEER": peer, "POMS_PEER_WGS": "8"})


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_distributed_kron_solve_gpu(world):
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    _launch("gpu_ksolve", world=world)


@pytest.mark.parametrize("world,nd,want", [(1, 3, (1, 1, 1)), (4, 3, (2, 2, 1)), (8, 3, (2, 2, 2)),
                                           (6, 2, (3, 2)), (12, 3, (3, 2, 2)), (7, 2, (7, 1))])
def test_dims_create(world, nd, want):
    assert dims_create(world, nd) == want


def test_cart_distribution_grid():
    """C-order ranks, per-axis blocks (slab_bounds) and neighbours of a 2x3x2 grid."""
    npts = (11, 13, 9)
    seen = np.zeros(npts, dtype=int)
    for r in range(12):
        d = CartDistribution(npts, (2, 3, 2), r)
        assert d.rank_of(d.coords) == r
        assert d.coords == (r // 6, (r // 2) % 3, r % 2)
        for ax in range(3):
            c = list(d.coords)
            if d.prev[ax] is not None:
                c[ax] -= 1
                assert d.prev[ax] == d.rank_of(c)
                c[ax] += 1
            if d.next[ax] is not None:
                c[ax] += 1
                assert d.next[ax] == d.rank_of(c)
            assert (d.prev[ax] is None) == (d.coords[ax] == 0)
            assert (d.next[ax] is None) == (d.coords[ax] == d.dims[ax] - 1)
        seen[tuple(slice(s, e) for s, e in zip(d.starts, d.ends))] += 1
    assert (seen == 1).all()
    with pytest.raises(ValueError):
        CartDistribution((3, 8), (4, 1), 3)   # 3 points over 4 ranks: rank 3 owns none


@pytest.mark.parametrize("dims", ["2x2x1", "1x2x2", "2x1x2", "2x2", "2x2x2"])
def test_four_rank_cart_exchange_and_block_apply_cpu(dims):
    """4 ranks (8 for 2x2x2: the triple corner of every interior block)."""
    world = int(np.prod([int(v) for v in dims.split("x")]))
    _launch("cart_cpu", world=world, extra_env={"POMS_TEST_CART_DIMS": dims})


@pytest.mark.gpu
@pytest.mark.parametrize("dims", ["2x2x1", "1x2x2", "2x2", "2x2x2"])
def test_four_rank_cart_operator_and_vcycle_gpu(dims):
    """spl Cart over a 2x2 process grid (axes 0/1, axes 1/2, and 2D) and 2x2x2 (8
    ranks on one GPU): device operator, sweeps, reductions, transfer and the
    V-cycle against the oracle."""
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    world = int(np.prod([int(v) for v in dims.split("x")]))
    _launch("cart_gpu", world=world, timeout=600, extra_env={"POMS_TEST_CART_DIMS": dims})


@pytest.mark.gpu
@pytest.mark.parametrize("dims", ["2x2", "2x2x1", "1x2x2", "2x2x2"])
def test_cart_kron_solve_and_pcg_glt_gpu(dims):
    """The Kronecker direct solve on Cart blocks (line-group transposes on every split
    axis) vs the oracle; pcg_glt on a 2x2 grid vs the reference's golden iterates."""
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    world = int(np.prod([int(v) for v in dims.split("x")]))
    _launch("cart_ksolve", world=world, timeout=600, extra_env={"POMS_TEST_CART_DIMS": dims})

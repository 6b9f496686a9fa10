"""Multi-process slab decomposition (world_size 2, gloo): one subprocess per rank."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

from poms_amd.dist import slab_bounds

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
    for r, (rc, out) in enumerate(outs):
        assert rc == 0, f"rank {r} failed (rc={rc}):\n{out[-4000:]}"
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
@pytest.mark.parametrize("world", [2, 3])
def test_two_rank_native_schedule_with_peers_gpu(world):
    """The production slab schedule (poms_op_run_dist: exchange, interior planes,
    both boundaries in one launch; lazy ring-slot norms; device-scalar pcg;
    restriction all-reduce through the library communicator) with REAL
    neighbours: the communicator's host transport moves the planes and sums over
    gloo, since RCCL cannot pair ranks that share one GPU."""
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    _launch("gpu", world=world, extra_env={"POMS_TEST_DEVRED": "1", "POMS_TEST_HOST_TRANSPORT": "1"})


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_distributed_kron_solve_gpu(world):
    import torch
    assert torch.cuda.device_count() >= 1, "GPU test selected but no GPU visible"
    _launch("gpu_ksolve", world=world)

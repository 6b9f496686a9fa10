"""The peer transport of the ghost exchange (``poms_comm_set_peer``, csrc/comm.hip):
one kernel on the communication stream that stores the boundary planes into the
receivers' mailboxes and copies its own mailboxes into the ghost planes, ordered by
per-workgroup flag slots.  Replaces `_update_ghost_regions_parallel`
(`pyccel/kron_product.py:21-41`).

Here on a one-rank loopback (the slab's own boundary planes come back into its
ghosts, as with RCCL's self-send): exact ghosts over repeated exchanges, workgroup
counts from 1 to 256, one-sided slabs, graph capture and replay, and the
distributed operator against the RCCL loopback bitwise.  Real neighbours (ranks in
separate processes sharing the GPU, IPC-mapped mailboxes) run in
``tests/test_dist.py`` with ``POMS_COMM_PEER=1``."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _comm(wgs):
    from poms_amd.dist import NativeComm
    torch.cuda.set_device(0)
    c = NativeComm.create_loopback()
    c.set_peer(True, wgs)
    return c


def _planes(n_loc, pad, pe, tag):
    data = torch.zeros((n_loc + 2 * pad, pe), dtype=torch.float64, device="cuda")
    for i in range(n_loc):
        data[pad + i] = torch.arange(pe, dtype=torch.float64, device="cuda") + 1e6 * (tag + 1) + 1e3 * i
    return data


def _check_ghosts(data, n_loc, pad, width, prev, nxt):
    h = data.cpu()
    for j in range(width):
        lo, hi = h[pad - width + j], h[pad + n_loc + j]
        if prev >= 0:   # loopback: the slab's own first planes
            assert torch.equal(lo, h[pad + j]), f"low ghost {j}"
        else:
            assert not bool(lo.any()), f"low ghost {j} written without a neighbour"
        if nxt >= 0:
            assert torch.equal(hi, h[pad + n_loc - width + j]), f"high ghost {j}"
        else:
            assert not bool(hi.any()), f"high ghost {j} written without a neighbour"


@pytest.mark.parametrize("wgs", [1, 7, 64, 256])
@pytest.mark.parametrize("pe", [16, 13, 515 * 528])   # 16-B vector and scalar copies, a headline plane
def test_peer_loopback_exchange(wgs, pe):
    from poms_amd import runtime as rt
    c = _comm(wgs)
    n_loc, pad, width = 7, 3, 3
    for rep in range(4):   # repeated exchanges: the flag slots count up
        data = _planes(n_loc, pad, pe, rep)
        c.halo_start(data, n_loc, pad, width, 0, 0, rt.stream_handle())
        c.halo_finish(rt.stream_handle())
        _check_ghosts(data, n_loc, pad, width, 0, 0)
    st = c.peer_status()
    assert st["active"] and not st["timed_out"], st


@pytest.mark.parametrize("prev,nxt", [(0, -1), (-1, 0)])
def test_peer_loopback_one_sided(prev, nxt):
    from poms_amd import runtime as rt
    c = _comm(16)
    n_loc, pad, width = 5, 2, 2
    for rep in range(3):
        data = _planes(n_loc, pad, 40, rep)
        c.halo_start(data, n_loc, pad, width, prev, nxt, rt.stream_handle())
        c.halo_finish(rt.stream_handle())
        _check_ghosts(data, n_loc, pad, width, prev, nxt)
    assert not c.peer_status()["timed_out"]


def test_peer_exchange_capture_and_replay():
    """The exchange is one kernel with device-side counters: captured once into a
    graph, every replay moves the CURRENT boundary planes."""
    c = _comm(32)
    n_loc, pad, width, pe = 6, 3, 3, 4096
    data = _planes(n_loc, pad, pe, 0)
    st = torch.cuda.Stream()
    c.peer_reserve(width * pe, 0, 0)   # mailboxes built outside the capture
    with torch.cuda.stream(st):   # warm-up (eager)
        c.halo_start(data, n_loc, pad, width, 0, 0, st.cuda_stream)
        c.halo_finish(st.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        c.halo_start(data, n_loc, pad, width, 0, 0, st.cuda_stream)
        c.halo_finish(st.cuda_stream)
    for rep in range(1, 5):
        data.copy_(_planes(n_loc, pad, pe, rep))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        _check_ghosts(data, n_loc, pad, width, 0, 0)
    assert not c.peer_status()["timed_out"]


@pytest.mark.parametrize("cells,rank", [(40, 1), (120, 1), (120, 0), (200, 2)])
def test_peer_loopback_operator_matches_rccl_loopback(cells, rank):
    """The distributed operator calls (interior planes beside the exchange, both
    boundaries after it) with the peer transport equal the RCCL transport's bitwise
    on the same loopback slab (both put the slab's own planes in its ghosts): apply,
    Jacobi sweep and its norm, residual, two sweeps from zero and their norms, apply
    + dot -- each call exchanging, twice over."""
    from poms_amd.dist import SlabDistribution
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    p = 3
    n = cells + p
    M, K = assemble_1d(uniform_knots(p, cells), p)
    outs = []
    for peer in (False, True):
        d = SlabDistribution.loopback(n, rank, 4)
        if peer:
            d.native.set_peer(True, 64)
        V = StencilVectorSpace([n] * 3, [p] * 3, align=True, dist=d)
        A = KronOperator.laplace(V, [M] * 3, [K] * 3)
        gen = torch.Generator(device="cuda").manual_seed(5)
        x, b = V.zeros(), V.zeros()
        V.interior(x._data).uniform_(-1, 1, generator=gen)
        V.interior(b._data).uniform_(-1, 1, generator=gen)
        res = []
        for _ in range(2):
            x._ghost_valid = False
            y = A.dot(x)
            xo = V.zeros()
            x._ghost_valid = False
            nrm = A.jacobi_sweep(b, x, xo, 2.0 / 3.0, want_norm=True)
            r = A.residual(b, xo)
            j0 = V.zeros()
            b._ghost_valid = False
            n0 = A.jacobi_from_zero(b, j0, 2.0 / 3.0, want_norm=True)
            x._ghost_valid = False
            ad = float(A.dot_inner(x, V.zeros(), device=True))
            torch.cuda.synchronize()
            res.append([V.interior(t._data).clone() for t in (y, xo, r, j0)] + [nrm, n0, ad])
        outs.append(res)
        if peer:
            st = d.native.peer_status()
            assert st["active"] and not st["timed_out"], st
    for a, b_ in zip(outs[0], outs[1]):
        for u, v in zip(a, b_):
            assert torch.equal(u, v) if isinstance(u, torch.Tensor) else u == v, (u, v)


def _loopback_op(cells=40, p=3, rank=1, world=4, peer=True):
    from poms_amd.dist import SlabDistribution
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    n = cells + p
    d = SlabDistribution.loopback(n, rank, world)
    if peer:
        d.native.set_peer(True, 32)
    M, K = assemble_1d(uniform_knots(p, cells), p)
    V = StencilVectorSpace([n] * 3, [p] * 3, align=True, dist=d)
    return d, V, KronOperator.laplace(V, [M] * 3, [K] * 3)


@pytest.mark.parametrize("peer", [True, False])
def test_peer_distributed_sweep_capture_and_replay(peer):
    """One distributed Jacobi sweep (exchange, interior launch, boundary launch on the
    communication stream, join) captured into a graph and replayed equals the eager
    call bitwise -- over the peer transport and over RCCL.  RCCL's grouped send/recv
    used to crash hipStreamEndCapture: torch's bundled HIP 7.0 runtime segfaults when
    RCCL P2P is captured on a stream forked from the capturing one; the library now
    queues captured RCCL calls on the capturing stream (round 6, tools/r06/graph_probe.cpp,
    profiles/r06/graph_probe/)."""
    d, V, A = _loopback_op(peer=peer)
    x, b = V.zeros(), V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    V.interior(b._data).uniform_(-1, 1)
    y_ref, y = V.zeros(), V.zeros()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        x._ghost_valid = False
        A.jacobi_sweep(b, x, y_ref, 2.0 / 3.0, want_norm=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        x._ghost_valid = False
        A.jacobi_sweep(b, x, y, 2.0 / 3.0, want_norm=False)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y._store, y_ref._store)
    assert not d.native.peer_status()["timed_out"]


@pytest.mark.parametrize("peer", [True, False])
def test_peer_pcg_graph_replay_matches_step_loop(monkeypatch, peer):
    """pcg + damped Jacobi on a loopback slab: the native loop's speculative calls
    replayed from its own captured graph (POMS_PCG_SPEC=1, POMS_PCG_GRAPH=2) give the
    step-by-step loop's iterates and info bitwise, and the graph was replayed -- over
    the peer transport and over RCCL."""
    from poms_amd import solvers
    d, V, A = _loopback_op(cells=48, peer=peer)
    b = V.zeros()
    V.interior(b._data).fill_(1.0)
    out = {}
    for mode in ("step", "graph"):
        monkeypatch.setenv("POMS_PCG_SPEC", "1" if mode == "graph" else "0")
        monkeypatch.setenv("POMS_PCG_GRAPH", "2" if mode == "graph" else "0")
        for _ in range(3):   # the graph run captures once, then replays
            x, info = solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=4)
        torch.cuda.synchronize()
        out[mode] = (x._data.clone(), dict(info))
    assert out["step"][1] == out["graph"][1]
    assert torch.equal(out["step"][0], out["graph"][0])
    st = A.spec_stats
    assert st["replays"] > 0, st
    assert not d.native.peer_status()["timed_out"]


def test_peer_mailboxes_not_rebuilt_after_capture():
    """Once an exchange has been captured, the mailboxes (whose raw addresses the graph
    holds) cannot be rebuilt or released: a larger reservation and set_peer(False)
    fail loudly instead of leaving the graph to write freed memory (advisor, round 5).
    The graph keeps working."""
    from poms_amd._lib import PomsError
    c = _comm(32)
    n_loc, pad, width, pe = 6, 3, 3, 1024
    data = _planes(n_loc, pad, pe, 0)
    st = torch.cuda.Stream()
    c.peer_reserve(width * pe, 0, 0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        c.halo_start(data, n_loc, pad, width, 0, 0, st.cuda_stream)
        c.halo_finish(st.cuda_stream)
    with pytest.raises(PomsError, match="captured"):
        c.peer_reserve(64 * width * pe, 0, 0)   # (past the 2^16-double minimum capacity)
    with pytest.raises(PomsError, match="captured"):
        c.set_peer(False)
    data.copy_(_planes(n_loc, pad, pe, 3))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    _check_ghosts(data, n_loc, pad, width, 0, 0)
    c.check()   # no exchange timed out

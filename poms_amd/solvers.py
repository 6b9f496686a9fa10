"""Krylov solver and smoothers of the V-cycle, with the reference's API.

Signatures, defaults, return conventions and stopping rules are those of
`sources/solvers.py`:

* ``pcg(A, psolve, b, x0=None, tol=1e-6, maxiter=100, verbose=False) -> (x, info)``
  (`sources/solvers.py:69-135`), ``info = {'niter', 'success', 'res_norm'}``;
  the stop test ``r.r < tol * ||r0||`` mixes squared and unsquared norms
  exactly as the reference does (:87, :113).
* ``damped_jacobi(A, b, x0=None, tol=1e-6, maxiter=10, verbose=False) -> x``
  (:167-235), omega = 2/3, stop when ``dr.dr < tol**2`` *after* the update.
* ``jacobi(A, b) -> x`` (:139-163).
* ``crl(A, b, x0=None, tol=1e-5, maxiter=1000, verbose=False) -> (x, info)``
  (:3-65): conjugate residual, stop when ``s.r < tol**2`` before the update.
* ``pcg_glt(A, M1, M2, b, x0=None, tol=1e-6, maxiter=100, verbose=False) -> (x, info)``
  (:239-306): the same PCG with the Kronecker direct solve
  ``kron_solve_par(M2, M1, r)`` as preconditioner (:258, :290), factorised once
  per (M2, M1) pair (``poms_amd.kron_solve``); :func:`pcg_kron` is its n-D form.

Differences that do not change results:
* the reference's discarded ``s = A.dot(r)`` (:109) is not computed;
* the per-element Python loop ``dr = omega*r/A[i,i,0,0]`` (:211-213) and the
  surrounding ``r = b - A.dot(x)``, ``x = x + dr``, ``dr.dot(dr)`` are one
  fused HIP kernel; the first sweep from ``x0 = None`` uses ``A.0 = 0``
  exactly and launches the diagonal scaling alone;
* with ``tol == 0`` the norms that can never stop the iteration are not
  computed (no host synchronisation);
* inside ``pcg`` with this module's ``damped_jacobi`` as ``psolve``, ``s.dot(r)``
  is accumulated by the final smoothing sweep (``poms_op_jacobi_sweep_dot``);
* ``q = A.dot(p)`` and ``p.dot(q)`` come from one pass (``poms_op_apply_dot``);
* from ``x0 = None`` sweeps 1 and 2 run as one pass over ``b``
  (``poms_op_jacobi_from_zero``); if the reference would stop after sweep 1,
  ``x1`` is formed separately and returned.

Inputs must be :mod:`poms_amd.stencil` device objects; there is no CPU path.
"""
from __future__ import annotations

import os
from math import sqrt

from .stencil import KronOperator, StencilVector

OMEGA = 2.0 / 3.0


def _check(A, b):
    if not isinstance(A, KronOperator) or not isinstance(b, StencilVector):
        raise TypeError("poms_amd solvers take a poms_amd.stencil.KronOperator and StencilVector "
                        "(device-resident); there is no CPU fallback")
    n = A.shape[0]
    assert A.shape == (n, n)
    assert b.shape == (n,)


def _print_header(title):
    print(title)
    print("+---------+---------------------+")
    print("+ Iter. # | L2-norm of residual |")
    print("+---------+---------------------+")


def pcg(A, psolve, b, x0=None, tol=1e-6, maxiter=100, verbose=False, *, _x0_owned=False):
    """Preconditioned conjugate gradient (`sources/solvers.py:69-135`).

    ``_x0_owned`` (internal: the V-cycle's own temporaries) lets the native loop
    iterate in x0's buffer instead of a copy of it -- the reference copies x0
    (`sources/solvers.py:82`); a caller that never reads x0 again loses nothing."""
    _check(A, b)
    V = b.space
    if (psolve is damped_jacobi and not verbose and V.lazy_reductions and A.apply_dot_supported
            and A.fused_dot_supported):
        if _native_ok(A, V):
            return _pcg_native(A, b, x0, tol, maxiter, _x0_owned)
        return _pcg_device(A, b, x0, tol, maxiter)
    ctx, lay = V.ctx, V.layout
    if x0 is None:
        x = V.zeros()
        r = V.empty().assign(b)          # r = b - A.0 = b exactly
    else:
        assert x0.shape == (A.shape[0],)
        x = x0.copy()
        r = A.residual(b, x)

    nrmr0 = sqrt(r.dot(r))
    s, sr = _psolve_dot(A, psolve, r)
    p = s
    q = V.empty()

    if verbose:
        _print_header("CG solver:")
        template = "| {:7d} | {:19.2e} |"

    k = 0
    nrmr = nrmr0 * nrmr0
    fused_pq = A.apply_dot_supported
    for k in range(1, maxiter + 1):
        if fused_pq:
            pq = A.dot_inner(p, q)       # q = A p and p.q in one pass
        else:
            A.dot(p, out=q)
            pq = p.dot(q)
        alpha = sr / pq
        nrmr = _pcg_r_update(V, alpha, r, q)        # r -= alpha q ; r.r
        if nrmr < tol * nrmr0:
            _vec(V, "poms_vec_axpby", 1.0, x, alpha, p, x)   # x += alpha p
            k -= 1
            break
        srold = sr
        s, sr = _psolve_dot(A, psolve, r)
        beta = sr / srold
        if p is s:
            raise RuntimeError("psolve returned its input buffer")
        _pcg_xp_update(V, alpha, beta, x, p, s)     # x += alpha p ; p = s + beta p  (old p, one pass)
        if verbose:
            print(template.format(k, sqrt(nrmr)))

    if verbose:
        print("+---------+---------------------+")
    info = {"niter": k, "success": nrmr < tol * nrmr0, "res_norm": sqrt(nrmr)}
    return x, info


def _pcg_device(A, b, x0, tol, maxiter):
    """pcg with damped_jacobi as psolve, scalars on the device.

    Same iterates and stopping rule as the host loop above (`sources/solvers.py:69-135`).
    alpha = s.r / p.q and beta = s.r / s.r_old are device tensors read by the
    update kernels (``poms_*_dev``); the host reads only r.r for the stop test,
    and only after the next preconditioner call is queued, so the device never
    idles waiting for the host.  If the test fires, that queued psolve(r) is
    discarded (the reference stops before computing it: results are identical).
    """
    import torch
    V = b.space
    if x0 is None:
        x = V.zeros()
        r = V.empty().assign(b)
    else:
        assert x0.shape == (A.shape[0],)
        x = x0.copy()
        r = A.residual(b, x)
    nrmr0 = sqrt(r.dot(r))
    s, sr = _damped_jacobi(A, r, want_dot=True, device_dot=True)
    if sr is None:
        sr = s.dot_device(r)
    p = s
    q = V.empty()
    k = 0
    nrmr = nrmr0 * nrmr0
    for k in range(1, maxiter + 1):
        pq = A.dot_inner(p, q, device=True)
        alpha = sr / pq
        nrm_dev = _pcg_r_update_dev(V, alpha, r, q)     # r -= alpha q ; r.r (device)
        pending = V.lazy_value(nrm_dev)
        srold = sr
        s_next, sr = _damped_jacobi(A, r, want_dot=True, device_dot=True)   # queued before the read
        if sr is None:
            sr = s_next.dot_device(r)
        nrmr = pending.value()
        if nrmr < tol * nrmr0:
            _vec_dev(V, "poms_vec_axpby_dev", torch.cat([torch.ones_like(alpha), alpha]), x, p, x)
            k -= 1
            break
        beta = sr / srold
        _pcg_xp_update_dev(V, torch.cat([alpha, beta]), x, p, s_next)
    info = {"niter": k, "success": nrmr < tol * nrmr0, "res_norm": sqrt(nrmr)}
    return x, info


def _native_ok(A, V) -> bool:
    """The whole pcg + damped-Jacobi loop runs in C (poms_pcg_jacobi) unless disabled
    (POMS_NATIVE_PCG=0), the space is a Cart block (its ghost exchange is the torch
    transport's) or a distributed space has no native communicator."""
    import os
    if os.environ.get("POMS_NATIVE_PCG", "1") == "0" or V.is_cart:
        return False
    return not V.is_distributed or V.dist.native is not None


def _pcg_native(A, b, x0, tol, maxiter, x0_owned=False):
    """pcg(A, damped_jacobi, b, x0, tol, maxiter) as one C call (``poms_pcg_jacobi``):
    the launches, device scalars and stop tests of :func:`_pcg_device`, bitwise the
    same iterates, without a Python round trip per launch."""
    import ctypes as C
    from . import _lib, runtime as rt
    V = b.space
    work = getattr(A, "_pcg_work", None)
    if work is None or work[0].space is not V:
        work = A._pcg_work = [V.empty() for _ in range(5)]
    # (x0 = None: the C loop zero-fills x's interior; empty() zeroes only the ghosts,
    # instead of a second full-storage fill)
    x = (V.empty() if os.environ.get("POMS_PCG_X_EMPTY", "1") != "0" else V.zeros()) if x0 is None else (x0 if x0_owned else x0.copy())
    if x0 is not None:
        assert x0.shape == (A.shape[0],)
    d = V.dist if V.is_distributed else None
    opts = _lib.PcgOpts(float(tol), int(maxiter), 1e-6, 10, OMEGA,
                        -1 if d is None or d.prev is None else int(d.prev),
                        -1 if d is None or d.next is None else int(d.next))
    info = _lib.PcgInfo()
    ptrs = (C.c_void_p * 5)(*[w._data.data_ptr() for w in work])
    _lib.call("poms_pcg_jacobi", A._h, d.native.h if d is not None else None,
              C.byref(opts), rt.ptr(b._data), rt.ptr(x._data), 0 if x0 is None else 1, ptrs, C.byref(info),
              rt.stream_handle())
    x._mark_written()
    for w in work:
        w._mark_written()
    A._calls += 1
    return x, {"niter": info.niter, "success": bool(info.success), "res_norm": info.res_norm}


def _vec_dev(V, name, ab, xv, yv, zv):
    from . import _lib, runtime as rt
    import ctypes as C
    _lib.call(name, V.ctx, C.byref(V.layout), rt.ptr(ab), rt.ptr(xv._data), rt.ptr(yv._data), rt.ptr(zv._data),
              rt.stream_handle())
    zv._mark_written()


def _pcg_r_update_dev(V, alpha, r, q):
    from . import _lib, runtime as rt
    import ctypes as C
    buf = V.scalar_buffer()
    _lib.call("poms_pcg_r_update_dev", V.ctx, C.byref(V.layout), rt.ptr(alpha), rt.ptr(r._data), rt.ptr(q._data),
              rt.ptr(buf), rt.stream_handle())
    r._mark_written()
    return V.device_sum(buf[0:1])


def _pcg_xp_update_dev(V, ab, x, p, s):
    from . import _lib, runtime as rt
    import ctypes as C
    _lib.call("poms_pcg_xp_update_dev", V.ctx, C.byref(V.layout), rt.ptr(ab), rt.ptr(x._data), rt.ptr(p._data),
              rt.ptr(s._data), rt.stream_handle())
    x._mark_written()
    p._mark_written()


def _psolve_dot(A, psolve, r):
    """``s = psolve(A, r)`` and ``s.dot(r)``; for this module's damped_jacobi the dot is
    accumulated by the last smoothing sweep itself (same values, one pass less)."""
    if psolve is damped_jacobi and A.fused_dot_supported:
        s, sr = _damped_jacobi(A, r, want_dot=True)
        if sr is not None:
            return s, sr
        return s, s.dot(r)
    s = psolve(A, r)
    return s, s.dot(r)


def _vec(V, name, a, xv, b, yv, zv):
    from . import _lib, runtime as rt
    import ctypes as C
    _lib.call(name, V.ctx, C.byref(V.layout), float(a), rt.ptr(xv._data), float(b), rt.ptr(yv._data),
              rt.ptr(zv._data), rt.stream_handle())
    zv._mark_written()


def _pcg_r_update(V, alpha, r, q) -> float:
    from . import _lib, runtime as rt
    import ctypes as C
    buf = V.scalar_buffer()
    _lib.call("poms_pcg_r_update", V.ctx, C.byref(V.layout), float(alpha), rt.ptr(r._data), rt.ptr(q._data),
              rt.ptr(buf), rt.stream_handle())
    r._mark_written()
    return V.global_dot(float(buf[0].item()))


def _pcg_xp_update(V, alpha, beta, x, p, s):
    from . import _lib, runtime as rt
    import ctypes as C
    _lib.call("poms_pcg_xp_update", V.ctx, C.byref(V.layout), float(alpha), float(beta), rt.ptr(x._data),
              rt.ptr(p._data), rt.ptr(s._data), rt.stream_handle())
    x._mark_written()
    p._mark_written()


def _pcg_update(V, alpha, x, p, r, q) -> float:
    from . import _lib, runtime as rt
    import ctypes as C
    buf = V.scalar_buffer()
    _lib.call("poms_pcg_update", V.ctx, C.byref(V.layout), float(alpha), rt.ptr(x._data), rt.ptr(p._data),
              rt.ptr(r._data), rt.ptr(q._data), rt.ptr(buf), rt.stream_handle())
    x._mark_written()
    r._mark_written()
    return V.global_dot(float(buf[0].item()))


def jacobi(A, b):
    """Point Jacobi ``x = b / diag(A)`` (`sources/solvers.py:139-163`)."""
    _check(A, b)
    x = b.space.empty()
    A.diag_scale(b, x, 1.0, want_norm=False)
    x.update_ghost_regions()
    return x


def damped_jacobi(A, b, x0=None, tol=1e-6, maxiter=10, verbose=False):
    """Weighted Jacobi, omega = 2/3 (`sources/solvers.py:167-235`); returns x."""
    return _damped_jacobi(A, b, x0, tol, maxiter, verbose)[0]


def _damped_jacobi(A, b, x0=None, tol=1e-6, maxiter=10, verbose=False, want_dot=False, device_dot=False):
    """damped_jacobi; with ``want_dot`` also returns ``x.b`` accumulated by the final
    sweep (None when the last sweep was not a full sweep); ``device_dot`` returns it
    as a device tensor and skips the last sweep's norm (it cannot change the result)."""
    _check(A, b)
    V = b.space
    omega = OMEGA
    tol_sqr = tol ** 2
    need = tol_sqr > 0.0 or verbose
    if verbose:
        _print_header("Damped Jacobi method:")
        template = "| {:7d} | {:19.2e} |"

    # Norms are read one sweep late: sweep k is queued before the host waits for
    # ||dr_{k-1}||^2 (copied to pinned memory), so the GPU never idles on the stop
    # test.  If sweep k-1 met it, x_{k-1} is returned -- sweep k wrote the other
    # buffer -- exactly the reference's result (`sources/solvers.py:219-222`).
    lazy = need and not verbose and V.lazy_reductions
    pending = None                      # (LazyScalar of sweep k-1, buffer holding x_{k-1})

    def settle(pend):
        if len(pend) == 3:          # sweeps 1 and 2 from zero: (norms, x2 buffer, b)
            lz, xbuf, rhs = pend
            if lz.value(0) < tol_sqr:
                x1 = V.empty()
                A.diag_scale(rhs, x1, omega)
                return True, x1
            return lz.value(1) < tol_sqr, xbuf
        lz, xbuf = pend
        return lz.value() < tol_sqr, xbuf

    k0 = 1
    if x0 is None and maxiter >= 2 and not verbose and not (want_dot and maxiter == 2) \
            and A.from_zero_supported:
        # k = 1, 2 from x = 0 in one pass over b (x1 = omega b / diag is formed on the fly)
        x = V.empty()
        res = A.jacobi_from_zero(b, x, omega, want_norm=need, lazy=lazy)
        if lazy:
            pending = (res, x, b)
        elif need:
            n1, n2 = res
            if n1 < tol_sqr:        # the reference stops after sweep 1: return x1 itself
                x1 = V.empty()
                A.diag_scale(b, x1, omega)
                return x1, None
            if n2 < tol_sqr:
                return x, None
        k0 = 3
    elif x0 is None:
        if maxiter < 1:
            return V.zeros(), None
        # k = 1 from x = 0:  r = b - A.0 = b,  dr = omega b / diag,  x = dr
        x = V.empty()
        nrmr = A.diag_scale(b, x, omega, want_norm=need, lazy=lazy)
        if lazy:
            pending = (nrmr, x)
        else:
            if need and nrmr < tol_sqr:
                if verbose:
                    print("+---------+---------------------+")
                return x, None
            if verbose:
                print(template.format(1, sqrt(nrmr)))
        k0 = 2
    else:
        assert x0.shape == (A.shape[0],)
        x = x0.copy()

    dot = None
    if maxiter >= k0:
        xn = V.empty()
        for k in range(k0, maxiter + 1):
            if want_dot and k == maxiter and device_dot and lazy:
                # the last sweep's stop test cannot change the result: no norm, dot on device
                nrmr, dot = A.jacobi_sweep(b, x, xn, omega, want_norm=False, want_dot=True, device_dot=True)
            elif want_dot and k == maxiter:   # the last sweep also forms x_out . b
                nrmr, dot = A.jacobi_sweep(b, x, xn, omega, want_norm=need, want_dot=True)
            else:
                nrmr = A.jacobi_sweep(b, x, xn, omega, want_norm=need, lazy=lazy)
            if pending is not None:         # stop test of the previous sweep
                done, xprev = settle(pending)
                pending = None
                if done:
                    return xprev, None
            x, xn = xn, x
            if want_dot and k == maxiter and device_dot and lazy:
                break
            if lazy and not (want_dot and k == maxiter):
                pending = (nrmr, x)
                continue
            if need and nrmr < tol_sqr:
                break
            if verbose:
                print(template.format(k, sqrt(nrmr)))
    if pending is not None and len(pending) == 3:
        # maxiter == 2 from zero: the loop never ran, so sweep 1's stop test is still
        # open -- if it fired, the reference returns x1 (`sources/solvers.py:219-222`)
        done, xprev = settle(pending)
        return xprev, None
    if pending is not None and not device_dot:   # the last sweep's test cannot change the result
        pending[0].value()
    if verbose:
        print("+---------+---------------------+")
    return x, dot


def pcg_kron(A, factors, b, x0=None, tol=1e-6, maxiter=100, verbose=False):
    """PCG preconditioned by ``X = (F0^-1 ⊗ F1^-1 [⊗ F2^-1]) R`` (``factors[d]`` acts on
    axis ``d``): the body of `sources/solvers.py:239-306` for any dimension."""
    from .kron_solve import solver_for
    ks = solver_for(b.space, tuple(factors))
    return pcg(A, lambda _A, r: ks.solve(r), b, x0=x0, tol=tol, maxiter=maxiter, verbose=verbose)


def pcg_glt(A, M1, M2, b, x0=None, tol=1e-6, maxiter=100, verbose=False):
    """GLT-preconditioned CG (`sources/solvers.py:239-306`).  As the reference, the
    preconditioner is ``kron_solve_par(M2, M1, r)`` (:258, :290): M2 acts on axis 0."""
    if b.space.ndim != 2:
        raise ValueError("pcg_glt is the 2D solver of the reference; use pcg_kron for other dimensions")
    return pcg_kron(A, (M2, M1), b, x0=x0, tol=tol, maxiter=maxiter, verbose=verbose)


def crl(A, b, x0=None, tol=1e-5, maxiter=1000, verbose=False):
    """Conjugate residual method (`sources/solvers.py:3-65`): device vectors, the
    operator's fused residual / apply kernels, in-place vector updates."""
    _check(A, b)
    V = b.space
    if x0 is None:
        x = V.zeros()
        r = V.empty().assign(b)          # b - A.0 = b exactly
    else:
        assert x0.shape == (A.shape[0],)
        x = x0.copy()
        r = A.residual(b, x)
    p = r.copy()
    q = A.dot(p)
    s = q.copy()
    sr = s.dot(r)
    tol_sqr = tol ** 2
    if verbose:
        _print_header("CG solver:")
        template = "| {:7d} | {:19.2e} |"
    k = 0
    for k in range(1, maxiter + 1):
        if sr < tol_sqr:
            k -= 1
            break
        alpha = sr / q.dot(q)
        x.axpby_(alpha, p, 1.0)          # x = x + alpha p
        r.axpby_(-alpha, q, 1.0)         # r = r - alpha q
        A.dot(r, out=s)
        srold = sr
        sr = s.dot(r)
        beta = sr / srold
        p.axpby_(1.0, r, beta)           # p = r + beta p
        q.axpby_(1.0, s, beta)           # q = s + beta q
        if verbose:
            print(template.format(k, sqrt(sr)))
    if verbose:
        print("+---------+---------------------+")
    info = {"niter": k, "success": sr < tol_sqr, "res_norm": sqrt(sr)}
    return x, info

#!/usr/bin/env python3
"""Host-loop latency probe for the 2D V-cycle's smoother (1027^2, p = 3):
pcg through the Python device loop vs the native C loop, with and without launch
timing, and a bare chain of Jacobi sweeps with / without a host read per sweep."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import numpy as np
    import torch
    from poms_amd import solvers
    from poms_amd.splines import assemble_1d, uniform_knots
    from poms_amd.stencil import KronOperator, StencilVectorSpace
    torch.cuda.set_device(0)
    out = {}
    for nd, N in ((2, 1024), (3, 64)):
        p = 3
        n = N + p
        M, K = assemble_1d(uniform_knots(p, N), p)
        V = StencilVectorSpace([n] * nd, [p] * nd, align=True)
        A = KronOperator.laplace(V, [M] * nd, [K] * nd)
        b = V.zeros().from_numpy(np.ones((n,) * nd))
        for native in ("0", "1"):
            os.environ["POMS_NATIVE_PCG"] = native
            for timing in (False, True):
                solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=10)
                torch.cuda.synchronize()
                if timing:
                    A.timing(True)
                t0 = time.perf_counter()
                for _ in range(3):
                    solvers.pcg(A, solvers.damped_jacobi, b, tol=1e-6, maxiter=10)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / 3
                A.timing(False)
                out[f"{nd}d_native{native}_timing{int(timing)}_ms_per_pcg"] = dt * 1e3
        x, y = V.zeros().from_numpy(np.ones((n,) * nd)), V.zeros()
        nb = V.scalar_buffer()
        for mode in ("nosync", "event", "item"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(100):
                A._run("jacobi", x, y, b=b, omega=2.0 / 3.0, norm_out=nb[0:1])
                x._ghost_valid = True
                if mode == "event":
                    ev = torch.cuda.Event()
                    ev.record()
                    ev.synchronize()
                elif mode == "item":
                    float(nb[0].item())
            torch.cuda.synchronize()
            out[f"{nd}d_sweep_{mode}_us"] = (time.perf_counter() - t0) / 100 * 1e6
        A.timing(True)
        for i in range(20):
            A._run("jacobi", x, y, b=b, omega=2.0 / 3.0, norm_out=nb[0:1])
        t, cnt, _ = A.timing_read("jacobi")
        A.timing(False)
        out[f"{nd}d_sweep_gpu_us"] = t / cnt * 1e6
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Time the Kronecker direct solve (csrc/kron_solve.hip) at a BASELINE size.

Per axis the algorithmic traffic is 32 B/DOF (read b, write y, read y, write x);
a 3D solve is 96 B/DOF.  Prints one JSON line per (n, bandwidth) case."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from poms_amd import _lib, runtime as rt  # noqa: E402
from poms_amd.kron_solve import KronSolver  # noqa: E402
from poms_amd.splines import collocation_cardinal_splines  # noqa: E402
from poms_amd.stencil import StencilVectorSpace  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 515
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    for label, p, F in (("collocation_p3", 3, None), ("band_kl3_ku3", 3, 3)):
        if F is None:
            C = collocation_cardinal_splines(p, n)
        else:
            rng = np.random.default_rng(0)
            C = np.triu(np.tril(rng.uniform(-1, 1, (n, n)), F), -F) + 4 * np.eye(n)
        V = StencilVectorSpace([n] * 3, [p] * 3, align=True)
        ks = KronSolver(V, [C, C, C])
        y = V.zeros()
        V.interior(y._data).copy_(torch.rand(V.local_npts, device=dev, dtype=torch.float64))
        x = V.empty()
        st = rt.stream_handle()
        res = {}
        for axis in (0, 1, 2):
            for _ in range(2):
                _lib.call("poms_kron_solve_axis", ks._h, axis, rt.ptr(y._data), rt.ptr(x._data), st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                _lib.call("poms_kron_solve_axis", ks._h, axis, rt.ptr(y._data), rt.ptr(x._data), st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            res[f"axis{axis}_us"] = round(us, 1)
            res[f"axis{axis}_GBps"] = round(32.0 * n ** 3 / us / 1e3, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ks.solve(y, out=x)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(json.dumps({"case": label, "n": n, "kl_ku": [ks.kl[0], ks.ku[0]], "solve_us": round(us, 1),
                          "solve_GBps_96B": round(96.0 * n ** 3 / us / 1e3, 1), **res}), flush=True)


if __name__ == "__main__":
    main()

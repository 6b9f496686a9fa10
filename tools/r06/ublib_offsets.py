#!/usr/bin/env python3
"""Round 6: does the placement of y relative to x change the L2 reuse of the march?

The memory-only march (tools/r06/ublib.hip, t16) read 8.1 B/DOF of x in the standalone
ubench (x, y consecutive hipMallocs) but 9.7 B/DOF on the library's arrays (x, b, y
from torch).  Here the same kernel runs on the library's x with y at chosen byte
offsets inside one raw buffer (every y keeps x's 128-B phase), one configuration
per process run, so that rocprofv3 --pmc passes can tell the configurations apart.

    python tools/r06/ublib_offsets.py <config>      (config -1: time every one)
"""
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

# y's offset past x's end, bytes (rounded to keep x's phase mod 128): "vec" = a separate
# library vector allocated right after x (no b in between)
CONFIGS = ["vec", 0, 4096, 65536, 1 << 20, (2 << 20) - 4096, 3 << 19, 8 << 20]


def main():
    import torch
    from poms_amd.stencil import StencilVectorSpace
    which = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    n = 515
    V = StencilVectorSpace([n] * 3, [3] * 3, align=True)
    x = V.zeros()
    V.interior(x._data).uniform_(-1, 1)
    yv = V.zeros()   # allocated right after x
    nbytes = x._store.numel() * 8
    raw = torch.zeros(nbytes // 8 + (16 << 20) // 8, dtype=torch.float64, device="cuda")
    ub = C.CDLL(str(ROOT / "tools/r06/ublib.so"))
    st = torch.cuda.current_stream()
    xp = x._data.data_ptr()
    res = {}
    for ci, cfg in enumerate(CONFIGS):
        if which >= 0 and ci != which:
            continue
        if cfg == "vec":
            yp = yv._data.data_ptr()
        else:
            base = raw.data_ptr() + cfg
            yp = base + ((xp - base) % 128)
        assert (yp - xp) % 128 == 0
        ts = []
        for _ in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert ub.ub_t16(C.c_void_p(xp), C.c_void_p(yp), 1, 0, C.c_void_p(st.cuda_stream)) == 0
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) * 1e3 for a, b in ts[2:]]
        res[str(cfg)] = {"median_us": round(statistics.median(t), 1), "min_us": round(min(t), 1),
                         "y_minus_x_mod_2MiB": (yp - xp) % (2 << 20), "x_mod_2MiB": xp % (2 << 20)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

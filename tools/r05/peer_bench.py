#!/usr/bin/env python3
"""Time one ghost exchange of the headline slab (3 planes of 515 x 528 doubles each
way, a 65-plane slab) on a one-rank loopback: RCCL self-send against the peer
kernel at several workgroup counts, fine-grained or plain mailboxes (events on
the caller's stream around halo_start + halo_finish).

    python tools/r05/peer_bench.py [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--pe", type=int, default=515 * 528)
    ap.add_argument("--planes", type=int, default=65)
    a = ap.parse_args()
    import torch
    from poms_amd.dist import NativeComm
    torch.cuda.set_device(0)
    pad = w = 3
    data = torch.zeros((a.planes + 2 * pad, a.pe), dtype=torch.float64, device="cuda")
    data[pad:pad + a.planes].uniform_(-1, 1)
    c = NativeComm.create_loopback()
    st = torch.cuda.current_stream()
    configs = [("rccl", 0, None)] + [("peer", g, "0") for g in (32, 64, 128, 256)] + [("peer", 64, "1")]
    for name, wgs, fine in configs:
        if name == "peer":
            os.environ["POMS_PEER_FINE"] = fine
            c.set_peer(False)
            c.set_peer(True, wgs)
        else:
            c.set_peer(False)
        ts = []
        for r in range(a.reps + 5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c.halo_start(data, a.planes, pad, w, 0, 0, st.cuda_stream)
            c.halo_finish(st.cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            if r >= 5:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ok = torch.equal(data[:pad], data[pad:2 * pad]) and torch.equal(data[-pad:], data[-2 * pad:-pad])
        st_ = c.peer_status() if name == "peer" else {}
        mb = 2 * w * a.pe * 8 / 1e6
        print(json.dumps({"transport": name, "wgs": wgs, "fine": fine, "median_us": round(statistics.median(ts), 1),
                          "min_us": round(min(ts), 1), "MB_each_way": mb, "ghosts_ok": bool(ok), **st_}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-XCD view of the raw workgroup stamps (tools/v5_stamps.py --raw): each XCD's
work / 32 CUs against its last end, the durations of its last 8 workgroups, and
workgroup duration against the number of workgroups running.

    python tools/r05/stamps_raw.py profiles/r05/sched/raw_sched.npz
"""
import numpy as np, sys
z = np.load(sys.argv[1])
for key in z.files:
    t0, t1, xcc, cu = z[key][:4]
    base = t0.min(); t0 = (t0 - base) / 100.0; t1 = (t1 - base) / 100.0
    n = len(t0); bx = np.arange(n); d = t1 - t0
    print(key)
    for x in range(8):
        sel = (bx & 7) == x
        print("  xcd %d work/32 %.0f last-end %.0f  last-start %.0f  dur med %.0f  tail-wg durs(last 8 started) %s" % (x, d[sel].sum() / 32, t1[sel].max(), t0[sel].max(), np.median(d[sel]), np.round(np.sort(d[sel][np.argsort(t0[sel])[-8:]])).astype(int).tolist()))
    # duration vs concurrency: number of wgs running at wg's midpoint
    mid = (t0 + t1) / 2
    conc = np.array([np.sum((t0 <= m) & (t1 >= m)) for m in mid])
    for lo, hi in ((0, 150), (150, 230), (230, 257)):
        s = (conc >= lo) & (conc < hi)
        if s.any(): print("  concurrency [%d,%d): %d wgs, median dur %.1f" % (lo, hi, s.sum(), np.median(d[s])))

#!/usr/bin/env python3
"""List-scheduling model of a v5 launch's grid at 515^3 (the J0 tile classes'
measured duration factors, 8 XCDs x 32 CUs, each XCD starting its contiguous range
in order with a 3 us gap per workgroup): the default order, longest-first within
each XCD's range, and weight-balanced ranges; then non-uniform axis-0 chunks.
Predicted 924 -> 852 us of span at 86-plane chunks (measured 885 -> 822 us in the
stamped build, profiles/r05/sched/).
"""
import heapq, numpy as np
T1n, T2n, N, P = 33, 5, 515, 3
F1 = {0: 1.21, 31: 1.20, 32: 1.54}
def f1(t): return F1.get(t, 1.0)
def f2(t): return 1.11 if t in (0, 4) else 1.0
PER_PLANE = 185.0 / (86 + 2 * P)
GAP = 3.0
def even(nch):
    base, r = divmod(N, nch); return [base + (1 if i < r else 0) for i in range(nch)]
def items(chunks):   # natural bid order, order 0: t2 fastest, then t1, chunk
    return [PER_PLANE * (npl + 2 * P) * f1(t1) * f2(t2) for ch, npl in enumerate(chunks) for t1 in range(T1n) for t2 in range(T2n)]
def run(queue, cus=32):
    free = [0.0] * cus; heapq.heapify(free); end = 0
    for w in queue:
        t = heapq.heappop(free) + GAP; heapq.heappush(free, t + w); end = max(end, t + w)
    return end
def natural(d):
    n = len(d); q, rr = n // 8, n % 8; out = []
    for x in range(8):
        lo = x * (q + 1) if x < rr else rr * (q + 1) + (x - rr) * q
        out.append(d[lo: lo + (q + 1 if x < rr else q)])
    return out
def balanced(d):   # contiguous ranges with equal weight
    c = np.cumsum(d); tot = c[-1]; cuts = [0]
    for x in range(1, 8): cuts.append(int(np.searchsorted(c, tot * x / 8)))
    cuts.append(len(d)); return [d[cuts[i]:cuts[i + 1]] for i in range(8)]
for nch in (6, 7, 9, 12):
    d = items(even(nch)); avg = sum(d) / 256
    r = {}
    r["nat"] = max(run(q) for q in natural(d))
    r["nat+lpt"] = max(run(sorted(q, reverse=True)) for q in natural(d))
    r["bal+lpt"] = max(run(sorted(q, reverse=True)) for q in balanced(d))
    print(nch, even(nch)[0], "avg %.0f" % avg, {k: round(v) for k, v in r.items()})
print("--- non-uniform chunks, LPT within balanced XCD ranges")
import itertools, random
def evalc(chunks):
    d = items(chunks); return max(run(sorted(q, reverse=True)) for q in balanced(d)), sum(d) / 256
best = []
for big in range(70, 130, 4):
    for nb in range(2, 7):
        rest = N - big * nb
        if rest <= 0: continue
        for small in range(10, 60, 4):
            ns = max(1, round(rest / small))
            sm = even_split = [rest // ns + (1 if i < rest % ns else 0) for i in range(ns)]
            ch = [big] * nb + sm
            s, avg = evalc(ch)
            best.append((s, avg, ch))
best.sort()
for s, avg, ch in best[:8]: print(round(s), round(avg), ch)

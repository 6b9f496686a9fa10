#!/usr/bin/env python3
"""Per-basic-block instruction classes of one kernel in a device .s file.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S kron_v5.hip -o v5.s
    python tools/isa_blocks.py v5.s <kernel-name-substring> [--body]

Prints, per block: label, instruction count, VALU (of which FP64, DPP, readlane /
writelane, 64-bit moves, cndmask), SALU, LDS, VMEM, waitcnt / barrier, and the
branch that ends it.  Used to count the hot path of the v5 march per plane.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\S*:\s*(;.*)?$", ln):
            on = sub in ln
            continue
        if on:
            if ln.startswith("\t.section") or re.match(r"^\.Lfunc_end", ln):
                break
            out.append(ln.rstrip("\n"))
    return out


def classify(op):
    c = Counter()
    c["all"] += 1
    if op.startswith("v_"):
        c["valu"] += 1
        if re.search(r"_f64", op):
            c["f64"] += 1
        if "dpp" in op:
            c["dpp"] += 1
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            c["lane"] += 1
        if op.startswith(("v_mov_b64", "v_pk_mov_b32")):
            c["mov64"] += 1
        if op.startswith("v_mov_b32") and "dpp" not in op:
            c["mov32"] += 1
        if op.startswith("v_cndmask"):
            c["cnd"] += 1
    elif op.startswith("s_waitcnt") or op.startswith("s_barrier"):
        c["wait"] += 1
    elif op.startswith("s_"):
        c["salu"] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
    elif op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        c["vmem"] += 1
    return c


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sub)
    blocks, cur, name = [], Counter(), "entry"
    term = ""
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):(.*)$", ln)
        if m:
            blocks.append((name, cur, term))
            name, cur, term = m.group(1) + m.group(2).replace("; %bb.", " bb").strip()[:40], Counter(), ""
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            if "Loop" in s:
                name += " [" + s[2:40] + "]"
            continue
        op = s.split()[0]
        cur.update(classify(op))
        if op.startswith("s_cbranch") or op.startswith("s_branch") or op.startswith("s_endpgm"):
            term = s[:60]
    blocks.append((name, cur, term))
    tot = Counter()
    keys = ["all", "valu", "f64", "dpp", "lane", "mov64", "mov32", "cnd", "salu", "lds", "vmem", "wait"]
    print("%-60s " % "block" + " ".join("%5s" % k for k in keys) + "  branch")
    for name, c, t in blocks:
        tot.update(c)
        print("%-60s " % name[:60] + " ".join("%5d" % c[k] for k in keys) + "  " + t)
    print("%-60s " % "TOTAL" + " ".join("%5d" % tot[k] for k in keys))


if __name__ == "__main__":
    main()

#!/bin/bash
# VGPR count and scratch bytes of every kron_v5_kernel build in poms_amd/_obj/kron_v5.hip.o
# (CPU-side check before a GPU run: a build with scratch would make the v5 launch refuse)
set -eu
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "${1:-poms_amd/_obj/kron_v5.hip.o}" $T/host.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$T/fb.bin --output=$T/dev.o --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/dev.o | python3 -c '
import sys, re
txt = sys.stdin.read()
for blk in re.split(r"\n\s*- \.agpr_count", txt)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if "kron_v5" not in name: continue
    v = re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)
    sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1)
    lds = re.search(r"\.group_segment_fixed_size:\s+(\d+)", blk).group(1)
    m = re.search(r"kron_v5_kernelILi(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d+)E", name)
    print("P=%s EPI=%s D=%s MODE=%s CP=%-3s vgpr %3s scratch %3s lds %6s %s" % (m.groups() + (v, sc, lds, name[-30:])))
'
rm -rf $T

#!/usr/bin/env python3
"""Register / scratch use of every kernel in a built object's device code.

    python tools/kernel_resources.py poms_amd/_obj/kron_v5.hip.o [name-substring ...]

Extracts the gfx950 code object from the object's .hip_fatbin section
(llvm-objcopy + clang-offload-bundler) and reads the AMDHSA metadata notes:
VGPRs, SGPRs, scratch bytes and spill counts per kernel; lists every kernel that
spills and the ones matching the substrings.
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = Path(d) / "fat.bin", Path(d) / "dev.co"
        subprocess.run([LLVM / "llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, Path(d) / "tmp.o"], check=True)
        subprocess.run([LLVM / "clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fat}", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([LLVM / "llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    out = []
    for k in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        g = lambda key: int(re.search(rf"\.{key}:\s+(\d+)", k).group(1))
        out.append((re.search(r"\.name:\s+(\S+)", k).group(1), g("vgpr_count"), g("sgpr_count"),
                    g("private_segment_fixed_size"), g("vgpr_spill_count"), g("sgpr_spill_count")))
    return out


def main():
    ks = kernels(sys.argv[1])
    subs = sys.argv[2:]
    spill = [k for k in ks if k[3] or k[4]]
    print(f"{len(ks)} kernels, {len(spill)} with scratch or VGPR spills")
    for k in spill:
        print("  SPILL", k[0][:110], "vgpr", k[1], "scratch", k[3], "vspill", k[4])
    for k in ks:
        if any(s in k[0] for s in subs):
            print(k[0][:110], "vgpr", k[1], "sgpr", k[2], "scratch", k[3], "sgpr_spill", k[5])


if __name__ == "__main__":
    main()

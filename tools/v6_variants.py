#!/usr/bin/env python3
"""Tuning builds of csrc/kron_v6.hip: each variant is the production source with
textual replacements, compiled and linked with the other objects of poms_amd/_obj
into poms_amd/exp/libv6_<name>.so (run with POMS_HIP_LIB=...).  Diagnostic
variants compute wrong results on purpose (timing only)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "poms_amd/csrc/kron_v6.hip"
VARIANTS = {
    "base": [],
    "allfast2": [("const bool fast2 = c0 >= tc.lo2 && cend <= tc.hi2;", "const bool fast2 = true;")],
    "nostore": [("(en && ((cok >> e) & 1)) ? voy + 8 * e : 0x7ffffff0", "(en && ((cok >> e) & 1) && vo[e] == 1.2345) ? voy + 8 * e : 0x7ffffff0")],
}


def build(name, reps):
    s = SRC.read_text()
    for a, b in reps:
        assert a in s, (name, a)
        s = s.replace(a, b)
    tmp = ROOT / "poms_amd/exp" / f"kron_v6_{name}.hip"
    tmp.parent.mkdir(exist_ok=True)
    tmp.write_text(s)
    obj = tmp.with_suffix(".o")
    fl = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-I", str(ROOT / "include"),
          "-I", str(ROOT / "poms_amd/csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", *fl, "-c", str(tmp), "-o", str(obj)], check=True)
    objs = [str(ROOT / "poms_amd/_obj" / (f + ".o")) for f in
            ["kron_fused.hip", "kron_dpp.hip", "kron_v4.hip", "kron_v5.hip", "vec_ops.hip", "transfer.hip",
             "kron_solve.hip", "stencil_general.hip", "comm.hip", "poms_abi.hip"]]
    out = ROOT / "poms_amd/exp" / f"libv6_{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), str(obj), *objs,
                    "-L/opt/rocm/lib", "-lrccl"], check=True)
    tmp.unlink()
    obj.unlink()
    print(out)


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        build(n, VARIANTS[n])

"""Build libpoms_hip.so in-tree with hipcc for gfx950 (no JIT cache, no setuptools).

The shared library is the C-ABI of ``include/poms_hip.h``; it is placed next to
this file so that it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB = HERE / "libpoms_hip.so"
OBJ = HERE / "_obj"
SOURCES = ["kron_fused.hip", "kron_dpp.hip", "kron_v4.hip", "kron_v5.hip", "kron_2d.hip", "vec_ops.hip", "transfer.hip", "kron_solve.hip", "stencil_general.hip", "comm.hip", "poms_abi.hip"]
ARCH = os.environ.get("POMS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _flags() -> list[str]:
    return [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
            "-Wno-unused-function", "-munsafe-fp-atomics"]


def _needs(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    # the source and the headers it includes by quoted name (csrc/ or include/)
    deps = [src]
    for line in src.read_text().splitlines():
        if line.startswith('#include "'):
            name = Path(line.split('"')[1]).name
            deps += [CSRC / name, HERE.parent / "include" / name]
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps if d.exists())


def _obj_name(s: str) -> str:
    return s + ".o"


def build(verbose: bool = False, force: bool = False, jobs: int = 4) -> Path:
    hipcc = _hipcc()
    OBJ.mkdir(exist_ok=True)
    todo = []
    for s in SOURCES:
        src, obj = CSRC / s, OBJ / _obj_name(s)
        if force or _needs(obj, src):
            todo.append((src, obj))

    def _compile(pair):
        src, obj = pair
        cmd = [hipcc, *_flags(), "-I", str(HERE.parent / "include"), "-c", str(src), "-o",
               str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
        return src.name

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for name in ex.map(_compile, todo):
            if verbose:
                print(f"compiled {name}", flush=True)
    objs = [str(OBJ / _obj_name(s)) for s in SOURCES]
    stamp = OBJ / "link.cfg"   # relink when the set of objects changes
    cfg = " ".join(objs)
    if force or todo or not LIB.exists() or not stamp.exists() or stamp.read_text() != cfg:
        tmp = LIB.with_suffix(".so.tmp")
        # librccl.so.1: at run time the one torch already loaded (same SONAME)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs,
               "-L/opt/rocm/lib", "-lrccl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        stamp.write_text(cfg)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))

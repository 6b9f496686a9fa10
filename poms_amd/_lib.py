"""ctypes binding of ``libpoms_hip.so`` (the C-ABI declared in ``include/poms_hip.h``).

This is the reference-side binding a maintainer would add: a
thin loader, one ``argtypes`` line per entry point, and a status check that
turns a non-zero return into ``PomsError(poms_last_error())``.  There is no
fallback: if the library is missing or cannot be loaded the import fails
loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("POMS_HIP_LIB", _HERE / "libpoms_hip.so"))
HEADER_PATH = _HERE.parent / "include" / "poms_hip.h"

FORM_SINGLE = 0
FORM_SUM = 1
LAYOUT_GHOST_DATA = 1


class PomsError(RuntimeError):
    """A libpoms_hip entry point returned a non-zero status."""


class Layout(C.Structure):
    _fields_ = [("n", C.c_int64 * 3), ("pads", C.c_int64 * 3), ("pitch", C.c_int64), ("flags", C.c_int64)]

    @classmethod
    def make(cls, n, pads, pitch=0, flags=0):
        lay = cls()
        for d in range(3):
            lay.n[d] = int(n[d])
            lay.pads[d] = int(pads[d])
        lay.pitch = int(pitch)
        lay.flags = int(flags)
        return lay


class PcgOpts(C.Structure):
    _fields_ = [("tol", C.c_double), ("maxiter", C.c_int), ("jtol", C.c_double), ("jmaxiter", C.c_int),
                ("omega", C.c_double), ("prev", C.c_int), ("next", C.c_int)]


class PcgInfo(C.Structure):
    _fields_ = [("niter", C.c_int), ("success", C.c_int), ("res_norm", C.c_double)]


_vp = C.c_void_p
_i64 = C.c_int64
_d = C.c_double
_i = C.c_int
_pp = C.POINTER(C.c_void_p)
_LP = C.POINTER(Layout)

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "poms_abi_version": [],
    "poms_last_error": [],
    "poms_device_count": [C.POINTER(_i)],
    "poms_ctx_create": [_i, _pp],
    "poms_ctx_destroy": [_vp],
    "poms_synchronize": [_vp, _vp],
    "poms_op_create": [_vp, _i, _LP, _i, _i, C.POINTER(C.c_void_p), _i64, _i64, _pp],
    "poms_op_destroy": [_vp],
    "poms_op_create_stencil": [_vp, _i, _LP, _vp, _i64, _i64, _pp],
    "poms_op_assemble_stencil": [_vp, _i, _LP, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _d, _i64,
                                 _pp],
    "poms_op_stencil_data": [_vp, _vp],
    "poms_op_set_chunk": [_vp, _i],
    "poms_op_set_tile_cols": [_vp, _i],
    "poms_op_set_variant": [_vp, _i],
    "poms_variant_built": [_i],
    "poms_diag_v5_stamps": [_vp, _i64],
    "poms_diag_v5_sched": [_i],
    "poms_op_get_variant": [_vp, C.POINTER(_i)],
    "poms_op_kernel_variant": [_vp, _i, C.POINTER(_i)],
    "poms_op_last_variant": [_vp, C.POINTER(_i)],
    "poms_op_spec_stats": [_vp, C.POINTER(_i)],
    "poms_vec_axpby_dev": [_vp, _LP, _vp, _vp, _vp, _vp, _vp],
    "poms_op_run_reduce": [_vp, _i, _d, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _i, _vp],
    "poms_op_run_reduce2": [_vp, _i, _d, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _i, _vp],
    "poms_comm_id_bytes": [],
    "poms_comm_unique_id": [C.c_char_p, _i],
    "poms_comm_create": [_i, C.c_char_p, _i, _i, _pp],
    "poms_comm_destroy": [_vp],
    "poms_comm_stream": [_vp, _pp],
    "poms_comm_create_host": [_i, _i, _i, _vp, _vp, _vp, _pp],
    "poms_comm_is_host": [_vp, C.POINTER(_i)],
    "poms_comm_host_attach_shm": [_vp, C.c_char_p, _i, C.POINTER(_i)],
    "poms_comm_uses_shm": [_vp, C.POINTER(_i)],
    "poms_halo_start": [_vp, _vp, _i64, _i64, _i, _i, _i, _i, _vp],
    "poms_halo_finish": [_vp, _vp],
    "poms_comm_set_peer": [_vp, _i, _i],
    "poms_comm_peer_reserve": [_vp, _i64, _i, _i],
    "poms_comm_peer_status": [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)],
    "poms_comm_check": [_vp],
    "poms_allreduce_sum": [_vp, _vp, _i64, _vp, _i],
    "poms_comm_slot": [_vp, _pp, C.POINTER(_i)],
    "poms_allreduce_to_host": [_vp, _i, _i, _vp, _vp],
    "poms_comm_wait": [_vp, _i],
    "poms_op_run_dist": [_vp, _vp, _i, _d, _vp, _vp, _vp, _vp, _i64, _i64, _i, _i, _i, _i, _i, _i, _i, _vp, _vp,
                         _i, _vp, C.POINTER(_i), _vp],
    "poms_copy_to_host_async": [_vp, _vp, _vp, _i64, _vp],
    "poms_pcg_r_update_dev": [_vp, _LP, _vp, _vp, _vp, _vp, _vp],
    "poms_pcg_xp_update_dev": [_vp, _LP, _vp, _vp, _vp, _vp, _vp],
    "poms_op_apply": [_vp, _vp, _vp, _i64, _i64, _vp],
    "poms_op_residual": [_vp, _vp, _vp, _vp, _i64, _i64, _vp],
    "poms_op_apply_dot": [_vp, _vp, _vp, _i64, _i64, _vp],
    "poms_op_apply_dot_supported": [_vp, C.POINTER(_i)],
    "poms_op_jacobi_sweep": [_vp, _d, _vp, _vp, _vp, _i64, _i64, _i, _vp],
    "poms_op_jacobi_sweep_dot": [_vp, _d, _vp, _vp, _vp, _i64, _i64, _i, _vp],
    "poms_op_fused_dot_supported": [_vp, C.POINTER(_i)],
    "poms_op_jacobi_from_zero": [_vp, _d, _vp, _vp, _i64, _i64, _i, _vp],
    "poms_op_from_zero_supported": [_vp, C.POINTER(_i)],
    "poms_op_sweep2_supported": [_vp, C.POINTER(_i)],
    "poms_op_jacobi3_from_zero": [_vp, _d, _vp, _vp, _vp, _vp],
    "poms_op_diag_scale": [_vp, _d, _vp, _vp, _i, _vp],
    "poms_op_last_partials": [_vp, C.POINTER(_i64)],
    "poms_op_set_ghost_corners": [_vp, _i],
    "poms_kron_dot_2d": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64],
    "poms_vec_axpby": [_vp, _LP, _d, _vp, _d, _vp, _vp, _vp],
    "poms_vec_scale": [_vp, _LP, _d, _vp, _vp, _vp],
    "poms_vec_fill": [_vp, _LP, _d, _vp, _vp],
    "poms_vec_zero_ghosts": [_vp, _LP, _vp, _vp],
    "poms_vec_dot": [_vp, _LP, _vp, _vp, _vp, _vp],
    "poms_pcg_update": [_vp, _LP, _d, _vp, _vp, _vp, _vp, _vp, _vp],
    "poms_pcg_r_update": [_vp, _LP, _d, _vp, _vp, _vp, _vp],
    "poms_pcg_xp_update": [_vp, _LP, _d, _d, _vp, _vp, _vp, _vp],
    "poms_reduce_partials": [_vp, _i64, _vp, _vp],
    "poms_reduce_partials_at": [_vp, _i64, _i64, _vp, _vp],
    "poms_transfer_create": [_vp, _i, _LP, _i64, _vp, _vp, C.POINTER(C.c_void_p), _pp],
    "poms_transfer_destroy": [_vp],
    "poms_restrict": [_vp, _vp, _vp, _vp],
    "poms_prolong_add": [_vp, _vp, _vp, _vp],
    "poms_transfer_set_operator": [_vp, _i, C.POINTER(C.c_void_p)],
    "poms_resid_restrict": [_vp, _vp, _vp, _vp, _vp],
    "poms_dense_matvec": [_vp, _i64, _vp, _vp, _vp, _vp],
    "poms_ksolve_create": [_vp, _i, _LP, _i64, C.POINTER(C.c_void_p), C.POINTER(_i64), C.POINTER(_i),
                           C.POINTER(_i), _pp],
    "poms_ksolve_create_global": [_vp, _i, _LP, C.POINTER(_i64), C.POINTER(C.c_void_p), C.POINTER(_i64),
                                  C.POINTER(_i), C.POINTER(_i), _pp],
    "poms_ksolve_destroy": [_vp],
    "poms_ksolve_info": [_vp, C.POINTER(_i)],
    "poms_ksolve_pivots": [_vp, _i, C.POINTER(_i)],
    "poms_kron_solve": [_vp, _vp, _vp, _vp],
    "poms_kron_solve_axis": [_vp, _i, _vp, _vp, _vp],
    "poms_kron_solve_axis0_dense": [_vp, _vp, _vp, _i64, _vp],
    "poms_kron_solve_lines_dense": [_vp, _i, _vp, _vp, _i64, _vp],
    "poms_kron_solve_bnd_2d": [_vp, _vp, _i64, _i, _i, _vp, _i64, _i, _i, _vp, _vp, _vp, _vp],
    "poms_pcg_jacobi": [_vp, _vp, C.POINTER(PcgOpts), _vp, _vp, _i, C.POINTER(C.c_void_p), C.POINTER(PcgInfo), _vp],
    "poms_op_timing": [_vp, _i, _i, _i, _i],
    "poms_op_timing_read": [_vp, _i, C.POINTER(_d), C.POINTER(_i64), C.POINTER(_i64)],
    "poms_kron_solve_bnd_3d": [_vp, _vp, _i64, _i, _i, _vp, _i64, _i, _i, _vp, _i64, _i, _i, _vp, _vp, _vp,
                               _vp],
}
_RESTYPES = {"poms_last_error": C.c_char_p}


def header_symbols(path: Path = HEADER_PATH) -> list[str]:
    """Every function the C header declares (used by the export test)."""
    text = path.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(poms_\w+)\s*\(", text, re.M)))


def _load() -> C.CDLL:
    # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Load
    # it first so that torch and libpoms_hip.so share ONE HIP runtime in the
    # process (device pointers and streams are passed between them).
    import torch  # noqa: F401
    if not LIB_PATH.exists():
        raise ImportError(
            f"libpoms_hip.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = C.CDLL(str(LIB_PATH))
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, C.c_int)
    return lib


lib = _load()


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib.poms_last_error().decode(errors="replace")
        raise PomsError(f"{what}: {msg}" if what else msg)


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args), name)

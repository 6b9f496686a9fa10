"""The C-ABI boundary without a GPU: library loads, every declared symbol is exported,
and calls that need no device report errors through the status/message protocol."""
import ctypes as C
import re
import subprocess

import pytest

from poms_amd import _lib


def test_header_declares_the_boundary():
    syms = _lib.header_symbols()
    assert len(syms) >= 25
    for must in ("poms_op_create", "poms_op_apply", "poms_op_residual", "poms_op_jacobi_sweep",
                 "poms_kron_dot_2d", "poms_restrict", "poms_prolong_add", "poms_resid_restrict",
                 "poms_transfer_set_operator", "poms_pcg_update"):
        assert must in syms


def test_every_header_symbol_is_exported():
    lib = _lib.lib
    missing = [s for s in _lib.header_symbols() if not hasattr(lib, s)]
    assert not missing, f"declared in include/poms_hip.h but not exported: {missing}"
    # the ctypes signature table covers the whole header, nothing more
    assert set(_lib._SIGS) == set(_lib.header_symbols())


def test_exports_are_plain_c():
    """No mangled C++ names in the dynamic symbol table for the poms_ entry points."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (poms_\w+)$", out, re.M))
    assert set(_lib.header_symbols()) <= exported


def test_abi_version_and_error_protocol():
    lib = _lib.lib
    assert lib.poms_abi_version() >= 1
    assert isinstance(lib.poms_last_error(), bytes)
    # null handles are rejected with a message, not a crash
    assert lib.poms_op_apply(None, None, None, 0, 0, None) != 0
    assert b"null" in lib.poms_last_error().lower() or lib.poms_last_error() != b""
    assert lib.poms_op_destroy(None) == 0
    assert lib.poms_transfer_destroy(None) == 0
    with pytest.raises(_lib.PomsError):
        _lib.call("poms_op_apply", None, None, None, 0, 0, None)


def test_gpu_required_calls_fail_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    rc = _lib.lib.poms_ctx_create(0, C.byref(h))
    assert rc != 0 and _lib.lib.poms_last_error()

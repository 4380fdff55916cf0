"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol declared in
include/dhcos.h, the ctypes table matches the header, and compute entry points fail loudly
(NativeError, no fallback) when no gfx950 device is present."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dhcos.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dh_[a-z_]+)\s*\(", txt)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ("dh_surface_price", "dh_surface_loss", "dh_price_pairs", "dh_cf", "dh_trunc_range",
              "dh_cos_coeffs", "dh_surface_loss_dev", "dh_surface_price_dev"):
        assert f in fns


def test_library_exports_every_header_symbol():
    from dhcos import _native
    lib = _native.load()
    for f in header_functions():
        assert hasattr(lib, f), f
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dh_[a-z_]+)\b", out))
    assert set(header_functions()) <= exported
    assert set(_native.SIGNATURES) == set(header_functions())


def test_header_constants_match_the_binding():
    """The Python binding's copies of the header's sizes: the request slots of dh_surface_fg_begin
    (DH_FG_SLOTS) and the sharded draw's state words (DH_GEN_LOC_WORDS)."""
    from dhcos import _native
    txt = open(HEADER).read()
    consts = dict((k, int(v)) for k, v in re.findall(r"#define (DH_[A-Z_]+) (\d+)", txt))
    assert consts["DH_FG_SLOTS"] == _native.FG_SLOTS
    assert consts["DH_GEN_LOC_WORDS"] == _native.GEN_LOC_WORDS


def test_library_is_gfx950_code_object():
    """The fat binary carries a gfx950 (MI355X) code object and nothing else."""
    from dhcos import _native
    data = open(_native.LIB_PATH, "rb").read()
    ids = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert ids == {b"gfx950"}, ids


def test_version_and_errors_without_device():
    from dhcos import _native
    lib = _native.load()
    assert lib.dh_version() >= 1
    if _native.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_native.NativeError):
        _native.Context(0)


def test_product_path_fails_loudly_without_device():
    from dhcos import DoubleHeston, NativeError, _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is present")
    dh = DoubleHeston(100, 100, 1.0, 0.05, 0.04, 2.0, 0.04, 0.3, -0.5, 0.04, 1.5, 0.04, 0.2, -0.3,
                      0.5, -0.05, 0.1)
    with pytest.raises(NativeError):
        dh.pricing()


def test_null_and_range_arguments_are_rejected():
    """Argument validation happens before any device work."""
    import ctypes as C
    from dhcos import _native
    lib = _native.load()
    assert lib.dh_ctx_create(0, None) == -1
    assert lib.dh_surface_price(None, None, None, 1, 128, 10.0, None) == -1
    assert b"null" in lib.dh_last_error()
    n = C.c_int32(-5)
    lib.dh_device_count(C.byref(n))
    assert n.value >= 0
    assert np.int8(1) == 1
    for setter in (lib.dh_ctx_set_tail_cut, lib.dh_ctx_set_exact, lib.dh_ctx_set_path):
        assert setter(None, 1) == -1                  # a null context, not a crash


def test_gen_assemble_arguments_are_rejected():
    """dh_gen_assemble (host code) validates its sizes and pointers."""
    from dhcos import _native
    lib = _native.load()
    assert lib.dh_gen_assemble(None, None, None, None, -1, 3, None, None, None) == -1
    assert lib.dh_gen_assemble(None, None, None, None, 4, 3, None, None, None) == -1
    assert lib.dh_gen_assemble(None, None, None, None, 0, 3, None, None, None) == 0


def test_comm_and_async_fg_arguments_are_rejected():
    """The communicator and the two-slot FD request validate their arguments before any device or
    RCCL work."""
    import ctypes as C
    from dhcos import _native
    lib = _native.load()
    out = C.c_void_p()
    uid = C.create_string_buffer(_native.COMM_ID_BYTES)
    assert lib.dh_comm_create(None, C.cast(uid, C.c_void_p), 1, 0, C.byref(out)) == -1
    assert lib.dh_comm_destroy(None) == 0
    assert lib.dh_comm_broadcast(None, None, 4, 0) == -1
    assert lib.dh_comm_allgather(None, None, 4, None) == -1
    best = C.c_int32(7)
    assert lib.dh_allgather_best(None, None, 1, 3, 0, 1, None, C.byref(best)) == -1
    assert lib.dh_surface_fg_begin(None, None, None, None, 1, 100.0, 0.05, 128, 10.0, 0) == -1
    assert lib.dh_surface_fg_end(None, None, 0, 0, None, None, None) == -1
    assert lib.dh_surface_fg_cancel(None, 0) == -1
    assert b"null" in lib.dh_last_error()


def test_price_cols_and_host_register_arguments_are_rejected():
    """dh_surface_price_cols and the page-locking pair validate their arguments before any device
    work; _native.pinned leaves an array it cannot register pageable (no device here) and never
    raises for it."""
    from dhcos import _native
    lib = _native.load()
    assert lib.dh_surface_price_cols(None, None, None, None, 0.03, 1, 128, 10.0, None) == -1
    assert b"null" in lib.dh_last_error()
    assert lib.dh_host_register(None, 64) == -1
    assert lib.dh_host_unregister(None) == -1
    a = np.ones(1000)
    with _native.pinned(a, None, np.empty(0)) as pin:
        if _native.device_count() == 0:
            assert pin._done == []                    # registration failed: left pageable
        a *= 2.0
    assert pin._done == [] and a[0] == 2.0            # whatever was registered is released

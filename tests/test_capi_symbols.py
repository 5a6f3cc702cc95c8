"""CPU-only: libdccrgx.so loads and exports exactly what include/dccrgx.h declares."""
import ctypes
import os
import re

from dccrg_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    txt = open(os.path.join(ROOT, "include", "dccrgx.h")).read()
    return sorted(set(re.findall(r"\b(dccrgx_\w+)\s*\(", txt)))


def test_header_matches_binding_table():
    assert declared() == sorted(_capi.SIGNATURES)


def test_library_exports_every_symbol():
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_loads_without_gpu():
    L = _capi.lib()
    assert L.dccrgx_version() == 1
    # pure host entry points work without a device
    out = ctypes.c_int32()
    ln = (ctypes.c_uint64 * 3)(100, 200, 300)
    _capi.check(L.dccrgx_max_possible_refinement_level(ln, ctypes.byref(out)))
    assert out.value == 13
    m = _capi.Mapping_t((ctypes.c_uint64 * 3)(10, 10, 1), 2, 0)
    last = ctypes.c_uint64()
    _capi.check(L.dccrgx_last_cell(ctypes.byref(m), ctypes.byref(last)))
    assert last.value == 100 + 800 + 6400

"""CPU-side checks of the C ABI library: it builds, loads and exports every
entry point declared in include/vibevoice_hip.h (no GPU compute here)."""
import ctypes
import os
import re

from vibevoice_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "vibevoice_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int|void)\s+(vv_\w+)\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared_symbols()
    assert "vv_lm_forward" in names and "vv_diffusion_sample" in names and "vv_codec_step" in names
    assert set(names) == {n for n, _, _ in _lib.EXPORTS}


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name


def test_config_struct_matches_header():
    # vv_config: 6 ints, 2 floats, 3 ints, 1 float, 1 int, 3 x int[8], 4 ints, 1 float, 2 ints
    assert ctypes.sizeof(_lib.VVConfig) == 4 * (6 + 2 + 3 + 1 + 1 + 24 + 4 + 1 + 2)


def test_create_rejects_bad_config():
    L = _lib.lib()
    c = _lib.VVConfig()
    c.head_dim = 64
    h = ctypes.c_void_p()
    assert L.vv_create(ctypes.byref(c), 0, ctypes.byref(h)) != 0
    assert b"head_dim" in L.vv_last_error()

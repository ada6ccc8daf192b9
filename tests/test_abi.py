"""The C-ABI library builds for gfx950, loads, and exports every symbol the header
declares (no compute call: this runs without a GPU)."""
import ctypes
import os
import re

from kmerpapa_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "kmerpapa_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(kp_[a-z_]+)\s*\(", txt)))


def test_header_symbols_exported():
    lib = engine.load()
    names = _declared()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/kmerpapa_hip.h but not exported"
    assert sorted(engine.EXPORTS) == names


def test_library_has_gfx950_code_object():
    data = open(engine.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_struct_layouts_match_header():
    # kp_group: 2 x int32 + 2 doubles + 8 doubles
    assert ctypes.sizeof(engine.KPGroup) == 4 + 4 + 8 + 8 + 8 * 8
    assert ctypes.sizeof(engine.KPPassStats) == 7 * 8

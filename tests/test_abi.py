"""The C-ABI shared library builds for gfx950, loads, and exports every entry point
declared in include/artes_amd.h (no compute calls: this runs without a GPU)."""

import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "artes_amd.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(artes_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("artes_grid_create", "artes_grid_destroy", "artes_run", "artes_run_device",
                     "artes_run_trace", "artes_last_kernel_ms", "artes_abi_version"):
        assert required in names


def test_library_exports_every_symbol():
    from artes_amd import engine

    lib = engine.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.artes_abi_version() == 1
    assert b"gfx950" in lib.artes_build_info()


def test_library_is_gfx950_code_object():
    from artes_amd import engine

    blob = open(engine.LIB_PATH, "rb").read()
    assert b".hip_fatbin" in blob or b"__hip_fatbin" in blob
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # offload bundle entry for gfx950


def test_struct_layouts_match_header():
    from artes_amd.abi import GridDesc, RunParams

    # 4 int32 + 8 pointers + 1 double ; 8 int32 + 9 doubles
    assert ctypes.sizeof(GridDesc) == 16 + 8 * 8 + 8
    assert ctypes.sizeof(RunParams) == 32 + 9 * 8


def test_product_path_does_not_import_oracle():
    import glob

    for f in glob.glob(os.path.join(ROOT, "artes_amd", "**", "*.py"), recursive=True):
        src = open(f).read()
        assert "import oracle" not in src and "from oracle" not in src, f

"""The C-ABI shared library builds for gfx950, loads, and exports every entry point
declared in include/artes_amd.h (no compute calls: this runs without a GPU)."""

import ctypes
import os
import re
import subprocess
import sys

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
                     "artes_run_trace", "artes_last_kernel_ms", "artes_abi_version", "artes_grid_thermal", "artes_run_flow", "artes_run_device_flow"):
        assert required in names


def test_library_exports_every_symbol():
    from artes_amd import engine

    lib = engine.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    from artes_amd.abi import ARTES_ABI_VERSION

    assert lib.artes_abi_version() == ARTES_ABI_VERSION == 6
    assert b"gfx950" in lib.artes_build_info()


def test_library_is_gfx950_code_object():
    from artes_amd import engine

    blob = open(engine.LIB_PATH, "rb").read()
    assert b".hip_fatbin" in blob or b"__hip_fatbin" in blob
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # offload bundle entry for gfx950


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirror (artes_amd/abi.py) has the C compiler's sizes and offsets."""
    import shutil
    import subprocess

    from artes_amd.abi import GridDesc, RunParams

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = []
    for cls, cname in ((GridDesc, "artes_grid_desc"), (RunParams, "artes_run_params")):
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "artes_amd.h"\nint main(void){' + "".join(lines)
                   + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cls, cname in ((GridDesc, "artes_grid_desc"), (RunParams, "artes_run_params")):
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_product_path_does_not_import_oracle():
    import glob

    for f in glob.glob(os.path.join(ROOT, "artes_amd", "**", "*.py"), recursive=True):
        src = open(f).read()
        assert "import oracle" not in src and "from oracle" not in src, f


def _undefined_symbols(path):
    import shutil
    import subprocess

    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--undefined-only", path], check=True, capture_output=True, text=True).stdout
    return {l.split()[-1].split("@")[0] for l in out.splitlines() if l.strip()}


def test_production_library_reads_no_environment():
    """The production library takes its schedule from artes_set_tuning alone: it imports no
    getenv / secure_getenv, so no ARTES_* variable in a user's shell can change the schedule or
    the engine.  The development build (libartes_hip_dev.so) does read them."""
    from artes_amd import engine

    und = _undefined_symbols(os.path.join(ROOT, "artes_amd", "lib", "libartes_hip.so"))
    assert not {"getenv", "secure_getenv"} & und
    dev = os.path.join(ROOT, "artes_amd", "lib", "libartes_hip_dev.so")
    if os.path.exists(dev):
        assert "getenv" in _undefined_symbols(dev)
    lib = engine.lib()
    assert b"development build" not in lib.artes_build_info()


def test_development_build_needs_opt_in(tmp_path):
    """A development build named by ARTES_LIB_PATH does not load without ARTES_DEV_LIB=1 (its
    schedule follows ARTES_* variables), and loads with it."""
    dev = os.path.join(ROOT, "artes_amd", "lib", "libartes_hip_dev.so")
    if not os.path.exists(dev):
        pytest.skip("development build not built")
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from artes_amd import engine\n"
            "try:\n    engine.lib(); print('loaded', engine.build_info())\n"
            "except engine.EngineUnavailable as e:\n    print('refused', e)\n") % ROOT
    env = {k: v for k, v in os.environ.items() if k != "ARTES_DEV_LIB"}
    env["ARTES_LIB_PATH"] = dev
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert out.stdout.startswith("refused"), out.stdout + out.stderr
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env=dict(env, ARTES_DEV_LIB="1"), timeout=300)
    assert out.stdout.startswith("loaded") and "development build" in out.stdout, out.stdout + out.stderr


def test_tuning_keys_without_device():
    """artes_set_tuning rejects a null grid; the key table is what the header documents."""
    import ctypes as C

    from artes_amd import engine

    lib = engine.lib()
    assert lib.artes_set_tuning(None, b"steps", 4) == -22
    assert lib.artes_get_tuning(None, b"steps") == -22
    txt = open(HEADER).read()
    for key in engine.TUNING_KEYS:
        assert key in txt, key
    assert C.sizeof(C.c_int64) == 8

"""Register budgets of the production kernels, read from the built library's gfx950 code
object (no GPU needed).

k_trace is issue-bound and runs 4 waves per SIMD (<= 128 VGPRs; the radial-only kernel 5,
<= 102); a register spill there costs several percent (round 3: a counted loop in the
list-queue flush spilled 12 VGPRs and cost ray3d 5.7 %), and the compiler's
allocation moves with small source changes.  This test pins the budgets so such a change
shows up in the CPU suite instead of only in a GPU timing run.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "artes_amd", "lib", "libartes_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels():
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(LIB) and os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("library or LLVM tools missing")
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "lib.so")
        shutil.copy(LIB, lib)
        subprocess.run([objdump, "--offloading", lib], cwd=d, check=True, capture_output=True)
        objs = [f for f in os.listdir(d) if "gfx950" in f]
        assert objs, "no gfx950 code object in the library"
        notes = subprocess.run([readelf, "--notes", os.path.join(d, objs[0])], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.match(r"\s*\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", line)
        if m and cur:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def _find(kernels, prefix):
    hits = {k: v for k, v in kernels.items() if k.startswith(prefix)}
    assert hits, f"no kernel {prefix}"
    return hits


def test_k_trace_budgets():
    ks = _kernels()
    # 3D grids (the bench and configs[3]): 4 waves per SIMD, no spills
    for name, r in _find(ks, "_ZN5artes7k_traceILb1ELb0ELi4ELb0E").items():
        assert r["vgpr_spill_count"] == 0, (name, r)
        assert r["vgpr_count"] <= 128, (name, r)
    # radial-only grids: a 5th wave per SIMD at <= 102 VGPRs
    for name, r in _find(ks, "_ZN5artes7k_traceILb0ELb0ELi4ELb0E").items():
        assert r["vgpr_spill_count"] == 0, (name, r)
        assert r["vgpr_count"] <= 102, (name, r)


def test_k_trace_step_counts():
    # steps per loop iteration: 10 on fine 3D and radial-only grids (8 before
    # round 6), 4 on coarse 3D grids -- both 3D instantiations and the radial-only one with 10 must
    # be in the library, with their global-table (GTAB) twins
    ks = _kernels()
    _find(ks, "_ZN5artes7k_traceILb1ELb0ELi4ELb0ELi10ELb0E")
    _find(ks, "_ZN5artes7k_traceILb1ELb0ELi4ELb0ELi4ELb0E")
    _find(ks, "_ZN5artes7k_traceILb0ELb0ELi4ELb0ELi10ELb0E")
    _find(ks, "_ZN5artes7k_traceILb1ELb0ELi4ELb0ELi10ELb1E")
    _find(ks, "_ZN5artes7k_traceILb0ELb0ELi4ELb0ELi10ELb1E")


def test_k_event_and_k_emit_budgets():
    ks = _kernels()
    for name, r in _find(ks, "_ZN5artes7k_event").items():
        assert r["vgpr_spill_count"] == 0, (name, r)
        if "Li768E" in name:   # one 768-thread block per CU: 3 waves per SIMD at <= 170 VGPRs
            assert r["vgpr_count"] <= 170, (name, r)
    for name, r in _find(ks, "_ZN5artes6k_emit").items():
        assert r["vgpr_spill_count"] == 0, (name, r)
    # the star-source emission on 3D grids: 4 waves per SIMD (kernel_event.hpp, STAR)
    for name, r in _find(ks, "_ZN5artes6k_emitILb1ELb0ELb1E").items():
        assert r["vgpr_count"] <= 128, (name, r)

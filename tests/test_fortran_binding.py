"""The reference-side binding: integration/artes_amd_c.f90 is the ISO_C_BINDING module a
maintainer of the Fortran reference would add, and integration/abi_probe.f90
a Fortran host that drives the C ABI the way `run` would (ARTES.f90:121-267).  Both are
compiled with amdflang against artes_amd/lib/libartes_hip.so.

CPU: the module's bind(C) structs have the C sizes, and the error paths (invalid grid,
null handle) return the documented negative codes.  GPU: the Fortran host transports a
batch and gets exactly the detector the ctypes host gets for the same packets."""

import math
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

AMDFLANG = shutil.which("amdflang") or ("/opt/rocm/bin/amdflang" if os.path.exists("/opt/rocm/bin/amdflang") else None)
need_flang = pytest.mark.skipif(AMDFLANG is None, reason="amdflang not installed")


def _build(tmp_path):
    lib = os.path.join(ROOT, "artes_amd", "lib")
    exe = tmp_path / "probe"
    subprocess.run([AMDFLANG, "-O1", "-J", str(tmp_path), "-o", str(exe),
                    os.path.join(ROOT, "integration", "artes_amd_c.f90"), os.path.join(ROOT, "integration", "abi_probe.f90"),
                    "-L" + lib, "-lartes_hip", "-Wl,-rpath," + lib], check=True, cwd=str(tmp_path))
    return exe


def _run(exe, n):
    out = subprocess.run([str(exe), str(n)], capture_output=True, text=True, timeout=300)
    kv = {}
    for line in out.stdout.splitlines():
        if "=" in line:
            k, v = line.split("=", 1)
            kv[k.strip()] = v.strip()
    return kv


@need_flang
def test_fortran_binding_compiles_and_reports_errors(tmp_path):
    from artes_amd.abi import ARTES_ABI_VERSION, GridDesc, RunParams
    import ctypes

    kv = _run(_build(tmp_path), 10)
    assert int(kv["abi_version"]) == ARTES_ABI_VERSION
    assert int(kv["sizeof_desc"]) == ctypes.sizeof(GridDesc)
    assert int(kv["sizeof_params"]) == ctypes.sizeof(RunParams)
    assert int(kv["bad_grid_rc"]) == -22 and "radial faces must increase" in kv["bad_grid_msg"]
    assert int(kv["null_grid_rc"]) == -22


@need_flang
@pytest.mark.gpu
def test_fortran_host_runs_the_engine(tmp_path, require_gpu):
    from artes_amd.abi import RunParams
    from artes_amd.engine import Grid

    n = 200000
    kv = _run(_build(tmp_path), n)
    assert int(kv["grid_rc"]) == 0 and int(kv["run_rc"]) == 0, kv
    assert int(kv["packets"]) == n and int(kv["errors"]) == 0
    # the same atmosphere and batch through the ctypes host
    nr = 4
    radial = 69911.0e3 + np.arange(nr + 1) * 25.0e3
    sm = np.zeros((180, 16, 1, 1, 1, nr))
    sm[:, 0] = 1.0 / (4.0 * math.pi)
    atm = dict(radial=radial, theta=np.array([0.0, 180.0]), phi=np.array([0.0]), wavelength=np.array([0.7]),
               scattering=np.full((1, 1, 1, nr), 1.0 / 100.0e3), absorption=np.zeros((1, 1, 1, nr)), scattermatrix=sm)
    g = Grid(atm, device=0)
    xm = 1.3 * radial[-1]
    p = RunParams(wl_index=0, nx=5, ny=5, photon_source=1, photon_scattering=1, phase_far=0, stellar_direction=0,
                  cell_depth=g.cell_depth(0), det_theta=math.pi / 2, det_phi=math.pi / 2, x_max=xm, y_max=xm,
                  fstop=1e-5, photon_minimum=1e-20, surface_albedo=0.0, theta_star=0.0, phi_star=0.0,
                  photon_emission=1, thermal_weight=1, ring=0, packet_moments=0, photon_bias=0.0)
    res = g.run(p, 0, n, 20171015)
    g.close()
    assert float(kv["detector_I"]) == pytest.approx(res.det[0, 0].sum(), rel=1e-14)
    assert int(kv["scatters"]) == res.counter("scatters")

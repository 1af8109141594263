"""The work-list invariants of the event engine (kernel_event.hpp, `Lists`: every live slot
named by exactly one list per stage, positions inside the pool, list modes consistent),
checked on the GPU by the ARTES_DEBUG build (artes_amd/lib/libartes_hip_debug.so, built by
__graft_entry__.build()) over schedules that stress the hand-off: tiny pools (hundreds of
iterations), the mirrored trace-list order, purely dynamic grabs, thermal + surface events
and a one-pixel detector.  A violation counts error 58 (ARTES_ERR_LISTS) and fails the run, as
do k_trace's trace-state checks (61: a pending bit other than the evaluated family's cleared;
62: a cell index outside the grid after a move or at a trace start);
the debug build must also transport exactly the release build's packets."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CASES = [
    ("ray3d", {}, {}),
    ("hg", {"ARTES_POOL": "3000", "ARTES_EMIT_FIRST": "1"}, {}),
    ("ray3d", {"ARTES_POOL": "5000", "ARTES_STATIC": "0", "ARTES_REFILL": "1"}, {}),
    ("thermal", {"ARTES_POOL": "4000"}, {"photon:source": "planet", "planet:surface_albedo": "0.5"}),
    ("ray3d", {"ARTES_POOL": "6000"}, {"detector:type": "phase"}),
    # the oblate star source: the reference's emission fails for every packet (errors 2, 31,
    # 43), so every event drops its packet -- the output trace list then needs twice the
    # slots (kernel_event.hpp, Lists (L2)); a small pool runs many such iterations
    ("oblate", {"ARTES_POOL": "2000"}, {}),
]

SCRIPT = r"""
import json, os, sys
sys.path.insert(0, {root!r})
from artes_amd import driver, synthetic
from artes_amd.engine import Grid
name, env, kv = json.loads(sys.argv[1])
os.environ.update(env)
atm = (synthetic.make_thermal(nr=8, ntheta=4, nphi=6, tau_abs=1.0, tau_sca=1.0) if name == "thermal"
       else synthetic.make_config("ray3d" if name == "oblate" else name,
                                  **({{}} if name not in ("ray3d", "oblate") else dict(nr=8, ntheta=8, nphi=8))))
cfg = driver.default_config()
for k, v in kv.items():
    cfg.apply(k, v)
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
g = Grid(atm, device=0, oblateness=0.1 if name == "oblate" else 0.0)
p = driver.run_params(cfg, det, 0, det_phi=0.7 if kv.get("detector:type") == "phase" else None, cell_depth=-1)
r = g.run(p, 0, 60000, 17)
print(json.dumps(dict(err=[int(e) for e in r.err], cnt=[int(c) for c in r.counters], det=float(r.det[0].sum()))))
"""


def _run(lib, case):
    env = dict(os.environ, ARTES_LIB_PATH=lib, ARTES_DEV_LIB="1")
    out = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT), json.dumps(case)], capture_output=True,
                         text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("build", ["debug", "nbf_debug"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_debug_build_list_invariants(require_gpu, case, build):
    """Both checked builds -- the shipping evaluation order and the nearest-pending-bound-first
    order (ARTES_NBF), which shares the pending-bit logic -- over the stress
    schedules (environment tuning: the debug builds are development builds), against the
    production library on its default schedule."""
    dbg = os.path.join(ROOT, "artes_amd", "lib", f"libartes_hip_{build}.so")
    rel = os.path.join(ROOT, "artes_amd", "lib", "libartes_hip.so")
    assert os.path.exists(dbg), "build() makes the ARTES_DEBUG library"
    d = _run(dbg, CASES[case])
    r = _run(rel, CASES[case])
    assert d["err"][58] == 0 and d["err"][57] == 0
    # k_trace trace-state checks: the evaluated family's pending bit is the one cleared, and
    # every cell index stays inside the grid (ARTES_ERR_PENDING, ARTES_ERR_CELL)
    assert d["err"][61] == 0 and d["err"][62] == 0
    assert d["cnt"] == r["cnt"] and d["cnt"][3] == 60000
    assert d["det"] == pytest.approx(r["det"], rel=1e-12)


@pytest.mark.skipif(os.environ.get("ARTES_FAULT_REPRO") != "1",
                    reason="opt-in (ARTES_FAULT_REPRO=1, after `make -C artes_amd/csrc nbf`): runs a build that "
                           "reconstructs a past device fault behind the debug guards")
def test_debug_build_catches_round2_fault(require_gpu):
    """The round-2 illegal access reconstructed in a CHECKED build (libartes_hip_nbf_old_debug:
    the nearest pending bound evaluated first with the round-2 clear of the lowest pending bit,
    DESIGN.md §4): the debug checks count the wrong clears (61) and the cell indices that then
    leave the grid (62), drop those packets before their out-of-range read, and fail the run;
    the shipping clear passes the same checks (test above)."""
    lib = os.path.join(ROOT, "artes_amd", "lib", "libartes_hip_nbf_old_debug.so")
    assert os.path.exists(lib), "`make -C artes_amd/csrc nbf` makes the reconstruction library"
    script = r"""
import json, sys
sys.path.insert(0, {root!r})
from artes_amd import driver, synthetic
from artes_amd.engine import EngineError, Grid
atm = synthetic.make_config("ray3d", share_matrix=True)
cfg = driver.default_config()
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
try:
    g.run(p, 0, 20000, 777)
    print(json.dumps(dict(failed=False)))
except EngineError as e:
    print(json.dumps(dict(failed=True, e61=int(e.err[61]), e62=int(e.err[62]))))
""".format(root=ROOT)
    out = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, ARTES_LIB_PATH=lib, ARTES_DEV_LIB="1"), cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["failed"] and r["e61"] > 0 and r["e62"] > 0, r

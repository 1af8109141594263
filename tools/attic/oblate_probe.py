"""The oblate-planet trajectory case of tests/test_gpu_parity.py under a given library, with
the engine's error counts (development tool; run the ARTES_DEBUG build to see the cell-index
checks, 61 / 62).  usage: ARTES_LIB_PATH=... python tools/oblate_probe.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, stats, synthetic  # noqa: E402
from artes_amd.engine import EngineError, Grid  # noqa: E402
from oracle.oracle import OracleGrid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20000
atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
cfg = driver.default_config()
g = Grid(atm, device=0, oblateness=0.1)
og = OracleGrid(atm, oblateness=0.1)
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
p = driver.run_params(cfg, det, 0, cell_depth=og.cell_depth(0))
try:
    r = g.run(p, 0, n, 31337)
    err, ok = r.err, True
except EngineError as e:
    err, ok = e.err, False
out = {"ok": ok, "err": {str(i): int(v) for i, v in enumerate(err) if v}}
o = og.run(p, 0, n, 31337, records=True)
out["oracle_err"] = {str(i): int(v) for i, v in enumerate(o[3]) if v}
print(json.dumps(out), flush=True)

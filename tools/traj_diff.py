"""Trajectory diff GPU vs oracle on the 8x8x8 ray3d parity grid: prints mismatching packets.
usage: python tools/traj_diff.py [oblateness] [on|off (photon scattering)] [packets]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, stats, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402
from oracle import oracle as oracle_mod  # noqa: E402

obl = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
scat = sys.argv[2] if len(sys.argv) > 2 else "on"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
cfg = driver.default_config()
grid = Grid(atm, device=0, oblateness=obl)
og = oracle_mod.OracleGrid(atm, oblateness=obl)
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
p = driver.run_params(cfg, det, 0, cell_depth=og.cell_depth(0))
p.photon_scattering = int(scat == "on")
gpu = grid.trace(p, 0, n, 31337)
ref = og.run(p, 0, n, 31337, records=True)[4]
same = stats.records_agree(gpu, ref)
print("agree", same.mean(), flush=True)
bad = np.nonzero(~same)[0]
for i in bad[:20]:
    print(i, "gpu", gpu[i, :4], "ref", ref[i, :4])

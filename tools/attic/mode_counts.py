"""Crossings per packet by trace kind, from a debug build of k_trace that counts them into
err[41] (first optical depth), err[42] (propagation after a scattering), err[43] (peel-off)
and err[51] (the propagation right after the forced first interaction) -- development tool:
ARTES_LIB_PATH=<debug lib> python tools/mode_counts.py [config] [packets]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "ray3d"
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10**7
cfg = driver.default_config()
atm = synthetic.make_config(name, share_matrix=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0), packet_moments=False)
r = g.run(p, 0, n, 7)
names = {41: "first optical depth", 51: "propagation after the forced interaction",
         42: "propagation after a scattering", 43: "peel-off"}
tot = 0.0
for k, nm in names.items():
    v = int(r.err[k]) / n
    tot += v
    print(f"{name}: {nm:44s} {v:8.2f} crossings/packet")
print(f"{name}: total {tot:.2f} (counter {r.counter('crossings') / n:.2f})")

"""One engine run for profiling: python tools/prof_one.py <config> <packets>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tuning  # noqa: E402
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "ray3d"
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10**7
cfg = driver.default_config()
if name == "cloudy":   # configs[3]'s shape (gas + Mie cloud, 16x6x6), a phase-curve call at 0.45 um
    import tempfile
    atm = synthetic.make_cloudy(tempfile.mkdtemp(), wavelength=(0.45, 0.7))
    cfg.apply("detector:type", "phase")
else:
    atm = synthetic.make_config(name, share_matrix=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
_tuning.apply(g)   # ARTES_* of the environment (artes_set_tuning)
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0), packet_moments=False)
w = g.run(p, 0, 10**5, 1)
r = g.run(p, 0, n, 2024)
print(name, n, "kernel ms %.1f -> %.3g pkt/s" % (g.last_kernel_ms(), n / (g.last_kernel_ms() * 1e-3)),
      "crossings (both runs) %d" % (r.counter("crossings") + w.counter("crossings")), flush=True)

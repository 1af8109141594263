"""Time the transport kernel for several event-deferral thresholds (development tool)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (one HIP runtime)
from artes_amd import driver, synthetic
from artes_amd.engine import Grid
cfg = driver.default_config()
for name in ["hg", "ray3d"]:
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    for d in [1, 4, 8, 16, 32, 48, 64]:
        os.environ["ARTES_DEFER"] = str(d)
        g.run(p, 0, 2 * 10**7, 1)
        ms = g.last_kernel_ms()
        print(name, "defer", d, "%.1f ms -> %.3g pkt/s" % (ms, 2e7 / ms * 1e3), flush=True)

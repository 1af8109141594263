"""Is k_trace VALU-bound?  Adds R.defer dependent FMAs per trace step (debug build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

cfg = driver.default_config()
n = 5 * 10**7
atm = synthetic.make_config("ray3d", share_matrix=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
g.set_profiling(True)
for spin in ("0", "0", "16", "48", "96", "192", "384"):
    os.environ["ARTES_DEFER"] = spin
    g.run(p, 0, n, 2024)
    kt = g.kernel_times()
    print(f"spin {spin}: total {g.last_kernel_ms():.1f} ms, k_trace {kt['trace'][0]:.1f} ms", flush=True)

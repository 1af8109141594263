"""Lane occupancy of k_trace (needs the -DARTES_DEBUG_LANES build via ARTES_LIB_PATH)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

cfg = driver.default_config()
for name in ("ray3d", "hg"):
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    for refill in ("16", "32", "48"):
        os.environ["ARTES_REFILL"] = refill
        n = 5 * 10**7
        r = g.run(p, 0, n, 2024)
        steps, lanes, refills = int(r.err[60]), int(r.err[61]), int(r.err[59])
        C = r.counter("crossings")
        print(f"{name} refill {refill}: {g.last_kernel_ms():.1f} ms, wave-steps {steps:.3e}, lanes/step {lanes / steps:.1f}, "
              f"crossings/wave-step {C / steps:.1f}, refills {refills:.3e} ({steps / refills:.1f} steps/refill)", flush=True)
    g.close()

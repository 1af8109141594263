"""Sweep the event engine's launch knobs (env ARTES_WPE / ARTES_REFILL / ARTES_POOL)."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 5 * 10**7
cfg = driver.default_config()
for name in ("ray3d", "hg"):
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    g.run(p, 0, 10**5, 1)
    combos = [dict(ARTES_LDS=l, ARTES_WPE=w, ARTES_REFILL=r, ARTES_STATIC=st)
              for l in ("0", "1") for w in ("4", "5") for r in ("32",) for st in ("0", "32")]
    combos += [dict(ARTES_LDS="1", ARTES_WPE="4", ARTES_REFILL=r, ARTES_STATIC="32") for r in ("16", "48")]
    for env in combos:
        os.environ.update(env)
        g.close()
        g = Grid(atm, 0)   # pool size is fixed at first use per grid
        g.run(p, 0, 10**5, 1)
        g.run(p, 0, n, 2024)
        ms = g.last_kernel_ms()
        print(f"{name} {env}: {ms:.1f} ms -> {n / (ms * 1e-3):.4g} pkt/s", flush=True)
    g.close()

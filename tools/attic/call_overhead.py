"""Fixed cost of one engine call (development tool): wall time of artes_run for small packet counts."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

cfg = driver.default_config()
atm = synthetic.make_config("ray3d", share_matrix=True)
g = Grid(atm, 0)
for nx in (25, 1):
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    if nx == 1:
        det = det._replace(nx=1, ny=1) if hasattr(det, "_replace") else det
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0), packet_moments=False)
    p.nx = nx; p.ny = nx
    for n in (0, 10**3, 10**4, 10**5, 10**6, 10**7):
        g.run(p, 0, n, 1)
        reps = 20 if n <= 10**5 else 5
        t = time.perf_counter()
        for _ in range(reps):
            g.run(p, 0, n, 1)
        dt = (time.perf_counter() - t) / reps
        print(f"detector {nx}x{nx} n={n:>9}: {dt * 1e3:8.3f} ms per call, last iterations {g.last_iterations() if hasattr(g, 'last_iterations') else '?'}", flush=True)
g.close()

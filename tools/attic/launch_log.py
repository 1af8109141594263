"""Per-launch kernel times over the iterations of one call (development tool): the cloudy
configs[3] phase calls at two detector azimuths and the bench's ray3d workload, each with
ARTES_LAUNCH_LOG so that every launch's time is written (kind 0 trace, 1 event, 2 emit, 3 aux).
usage: python tools/launch_log.py <out dir> [packets]"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

out = sys.argv[1]
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10**8
os.makedirs(out, exist_ok=True)


def run(grid, p, n, tag):
    grid.set_profiling(True)
    grid.run(p, 0, 10**5, 1)
    grid.kernel_times()
    log = os.path.join(out, tag + ".txt")
    if os.path.exists(log):
        os.remove(log)
    r = grid.run(p, 0, n, 2024)
    os.environ["ARTES_LAUNCH_LOG"] = log
    kt = grid.kernel_times()
    del os.environ["ARTES_LAUNCH_LOG"]
    c = r.counters.astype(np.float64)
    print(f"{tag}: {grid.last_kernel_ms():.1f} ms, C/pkt {c[0] / n:.1f} S/pkt {c[1] / n:.2f} "
          + " ".join(f"{k} {v[0]:.1f} ({v[1]})" for k, v in kt.items() if v[1]), flush=True)
    grid.set_profiling(False)


wl = tuple(np.round(np.linspace(0.45, 0.95, 50), 6))
atm = synthetic.make_cloudy(os.path.join(tempfile.mkdtemp(), "cloudy50"), wavelength=wl)
g = Grid(atm, device=0)
cfg = driver.default_config()
cfg.apply("detector:type", "phase")
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
phis = driver.phase_angles()
for k in (0, 24, 36):
    p = driver.run_params(cfg, det, 0, det_phi=phis[k], cell_depth=g.cell_depth(0), packet_moments=False)
    run(g, p, n, f"cloudy_phase{k}")
g.close()
atm = synthetic.make_config("ray3d", nr=32, ntheta=32, nphi=32)
g = Grid(atm, device=0)
cfg = driver.default_config()
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0), packet_moments=False)
run(g, p, 3 * n, "ray3d")
g.close()

"""Throughput of the heterogeneous (gas + Mie cloud, per-cell matrix ids) path (development tool).
usage: python tools/cloudy_perf.py [n_packets]"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**8
cfg = driver.default_config()
with tempfile.TemporaryDirectory() as d:
    t = time.time()
    atm = synthetic.make_cloudy(d)
    print(f"cloudy atmosphere built in {time.time() - t:.1f} s", flush=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
print(f"distinct matrices {g.num_matrices()}", flush=True)
g.set_profiling(True)
for wl in range(len(atm["wavelength"])):
    p = driver.run_params(cfg, det, wl, cell_depth=g.cell_depth(wl), packet_moments=False)
    g.run(p, 0, 10**5, 1)
    g.kernel_times()
    r = g.run(p, 0, n, 2024)
    kt = g.kernel_times()
    ms = g.last_kernel_ms()
    print(f"  wl {atm['wavelength'][wl]:.2f} um: {ms:.1f} ms -> {n / ms * 1e3:.4g} pkt/s  C/pkt {r.counter('crossings') / n:.1f} "
          f"S/pkt {r.counter('scatters') / n:.2f}  " + " ".join(f"{k} {v[0]:.1f}" for k, v in kt.items() if v[1]), flush=True)
g.close()

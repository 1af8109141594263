"""Tail parking (k_trace) development check: trajectory agreement with every trace parked
after each step, then throughput for several thresholds.
usage: python tools/park_check.py [n_packets]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402
from oracle.oracle import OracleGrid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 4 * 10**8
cfg = driver.default_config()
for name, atm, kv in (("ray3d", synthetic.make_config("ray3d", share_matrix=True), {}),
                      ("thermal", synthetic.make_thermal(nr=10, ntheta=6, nphi=8, tau_abs=1.0, tau_sca=2.0),
                       {"photon:source": "planet"})):
    c = driver.default_config()
    for k, v in kv.items():
        c.apply(k, v)
    det = driver.detector_geometry(c, atm["radial"][-1])
    g = Grid(atm, 0)
    p = driver.run_params(c, det, 0, cell_depth=-1)
    ref = OracleGrid(atm).run(p, 0, 20000, 777, records=True)[4]
    for env in ({"ARTES_PARK": "0"}, {"ARTES_PARK": "64", "ARTES_PARK_MIN": "1"}):
        os.environ.update(env)
        rec = g.trace(p, 0, 20000, 777)
        same = (np.isclose(rec[:, 0], ref[:, 0], rtol=1e-9, atol=1e-300) & (rec[:, 1] == ref[:, 1])
                & (rec[:, 2] == ref[:, 2]) & (rec[:, 3] == ref[:, 3]))
        print(f"{name} {env}: trajectory agreement {same.mean():.5f}", flush=True)
    os.environ.pop("ARTES_PARK_MIN", None)
    if name != "ray3d":
        continue
    g.set_profiling(True)
    for park in ("0", "8", "16", "24", "32"):
        os.environ["ARTES_PARK"] = park
        g.run(p, 0, 10**5, 1)
        g.kernel_times()
        g.run(p, 0, n, 2024)
        kt = g.kernel_times()
        ms = g.last_kernel_ms()
        print(f"  {name} park {park}: {ms:.1f} ms -> {n / ms * 1e3:.4g} pkt/s  "
              + " ".join(f"{k} {v[0]:.1f}/{v[1]}" for k, v in kt.items() if v[1]), flush=True)
    g.close()

"""Quick GPU sanity + timing run (development tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from artes_amd import driver, synthetic
from artes_amd.engine import Grid
from oracle.oracle import OracleGrid

cfg = driver.default_config()
for name in ["iso", "hg", "ray3d"]:
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    t = time.time(); g = Grid(atm, 0); print(name, "grid create %.2fs nmat %d" % (time.time() - t, g.num_matrices()), flush=True)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    n = 20000
    rec = g.trace(p, 0, n, 777)
    o = OracleGrid(atm)
    ref = o.run(p, 0, n, 777, records=True)[4]
    same = np.isclose(rec[:, 0], ref[:, 0], rtol=1e-9, atol=1e-300) & (rec[:, 1] == ref[:, 1]) & (rec[:, 3] == ref[:, 3])
    print("  per-packet agreement %.5f  (scat %.3f vs %.3f, cross %.2f vs %.2f)" % (same.mean(), rec[:, 1].mean(), ref[:, 1].mean(), rec[:, 2].mean(), ref[:, 2].mean()), flush=True)
    bad = np.where(~same)[0][:5]
    for b in bad:
        print("    mismatch", b, rec[b], ref[b])
    for n in [10**6, 10**7, 10**8]:
        t = time.time(); r = g.run(p, 0, n, 2024); dt = time.time() - t
        ms = g.last_kernel_ms()
        E = driver.package_energy(cfg, 0.7e-6, atm["radial"][-1], n, det.det_phi)
        ph = driver.photometry(driver.scale_detector(r.det[:3], E))
        print("  n=%.0e wall %.3fs kernel %.1f ms -> %.3g pkt/s  I %.6g Q %.6g U %.3g  C/pkt %.2f S/pkt %.3f err %s" % (
            n, dt, ms, n / (ms * 1e-3), 1e-6 * ph[0], 1e-6 * ph[2], 1e-6 * ph[4], r.counter("crossings") / n, r.counter("scatters") / n,
            {i: int(e) for i, e in enumerate(r.err) if e}), flush=True)
    g.close()

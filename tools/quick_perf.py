"""Quick throughput + trajectory agreement check (development tool).
usage: python tools/quick_perf.py [n_packets] [ENV=VAL ...]  (each ENV set is one variant)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from artes_amd import driver, stats, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tuning  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 5 * 10**7
variants = [dict(kv.split("=", 1) for kv in v.split(",")) if v else {} for v in (sys.argv[2:] or [""])]
cfg = driver.default_config()
check = os.environ.get("QP_CHECK", "1") == "1"
if check:
    from oracle.oracle import OracleGrid
for name in ("ray3d", "hg", "iso"):
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    _tuning.apply(g)   # ARTES_* of the environment (artes_set_tuning)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    if check:
        rec = g.trace(p, 0, 20000, 777)
        ref = OracleGrid(atm).run(p, 0, 20000, 777, records=True)[4]
        same = stats.records_agree(rec, ref)
        print(f"{name}: trajectory agreement {same.mean():.5f}", flush=True)
    g.set_profiling(True)
    for env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        tv = _tuning.apply(g, env)
        # QP_MOMENTS=0: production configuration without packet-level moments
        pv = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0),
                               packet_moments=os.environ.get("QP_MOMENTS", "1") == "1")
        g.run(pv, 0, 10**5, 1)
        g.kernel_times()
        g.run(pv, 0, n, 2024)
        kt = g.kernel_times()
        ms = g.last_kernel_ms()
        print(f"  {name} {env}: {ms:.1f} ms -> {n / ms * 1e3:.4g} pkt/s  "
              + " ".join(f"{k} {v[0]:.1f}" for k, v in kt.items() if v[1]), flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        if tv:
            g.set_tuning(**{k: None for k in tv})
            _tuning.apply(g)
    g.close()

"""k_trace blocks-per-CU sweep (ARTES_TRACE_BPC) at the default launch knobs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

cfg = driver.default_config()
n = 5 * 10**7
for name in ("ray3d", "hg"):
    atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    os.environ["ARTES_VERBOSE"] = "1"
    g.run(p, 0, 10**5, 1)
    os.environ.pop("ARTES_VERBOSE")
    for wpe in ("4", "5"):
        for bpc in ("", "2", "3", "4", "5", "6", "8"):
            os.environ["ARTES_WPE"] = wpe
            if bpc:
                os.environ["ARTES_TRACE_BPC"] = bpc
            else:
                os.environ.pop("ARTES_TRACE_BPC", None)
            g.run(p, 0, n, 2024)
            print(f"{name} wpe {wpe} bpc {bpc or 'api'}: {g.last_kernel_ms():.1f} ms -> {n / g.last_kernel_ms() * 1e3:.4g} pkt/s", flush=True)
    g.close()

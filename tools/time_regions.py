"""Where a k_trace wave's time goes, region by region (needs the -DARTES_DEBUG_TIMING build via
ARTES_LIB_PATH: per wave, the shader-clock cycles of each region of the loop, summed over waves).
usage: python tools/time_regions.py [packets] [ENV=VAL,ENV=VAL ...]   (one variant per argument)
LS_WORKLOAD=cloudy: the configs[3] cloudy atmosphere (0.45 micron, the phase mode's 1-pixel
detector) instead of ray3d.  The clock reads perturb the loop by a few per cent."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

REGIONS = ["parked blocks (first interaction, interaction + peel set-up)", "refill (append, take, record loads, set-up)",
           "evaluation (all families)", "step (choice, next cell, move)", "chain end (record store, queue flush)"]

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 5 * 10**7
variants = [dict(kv.split("=", 1) for kv in v.split(",")) if v else {} for v in (sys.argv[2:] or [""])]
cfg = driver.default_config()
name = os.environ.get("LS_WORKLOAD", "ray3d")
if name == "cloudy":
    import tempfile

    atm = synthetic.make_cloudy(os.path.join(tempfile.mkdtemp(), "cloudy"), wavelength=(0.45,))
    cfg.apply("detector:type", "phase")
else:
    atm = synthetic.make_config(name, share_matrix=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])
g = Grid(atm, 0)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tuning
_tuning.apply(g)
g.set_profiling(True)
p = driver.run_params(cfg, det, 0, det_phi=1e-5 if name == "cloudy" else None, cell_depth=g.cell_depth(0),
                      packet_moments=False)
for env in variants:
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    g.run(p, 0, 10**5, 1)
    g.kernel_times()
    r = g.run(p, 0, n, 2024)
    kt = g.kernel_times()
    e = [int(r.err[k]) for k in range(28)]
    total, iters = e[7], max(e[6], 1)
    C = r.counter("crossings")
    print(f"{name} {env}: {g.last_kernel_ms():.1f} ms, k_trace {kt['trace'][0]:.1f} ms, wave-iterations {iters:.3e}, "
          f"crossings/wave-iteration {C / iters:.1f}, wave cycles per iteration {total / iters:.0f}", flush=True)
    split = [e[0], e[1], e[2], e[3] - e[2], e[4]]
    for lab, v in zip(REGIONS, split):
        print(f"    {lab:62s} {v / total:6.3f}  ({v / iters:7.0f} cycles per iteration)")
    rest = total - sum(split)
    print(f"    {'outside the loop regions (loop head, exit, staging)':62s} {rest / total:6.3f}")
    subs = [("  of the parked blocks: the first interaction", e[13]), ("  of the parked blocks: interaction + peel set-up", e[14]),
            ("  of the refill: append (late list appends)", e[8]), ("  of the refill: take (cursor, chunk grabs)", e[9]),
            ("  of the refill: list entry load", e[10]), ("  of the refill: record load", e[11]),
            ("  of the refill: trace set-up", e[12]), ("  of the evaluation: the batched theta form", e[5])]
    for lab, v in subs:
        print(f"    {lab:62s} {v / total:6.3f}  ({v / iters:7.0f} cycles per iteration)")
    if e[27]:   # k_event's regions (kernel_event.hpp, ev_tick)
        ev = e[27]
        print(f"  k_event: {e[26]:.3e} wave-events, {ev / max(e[26], 1):.0f} wave cycles per event: latch copy (the prefetched "
              f"record's wait) {e[20] / ev:.3f}, event {e[21] / ev:.3f} (peel {e[22] / ev:.3f}, angle sampling {e[23] / ev:.3f}, "
              f"rest of the scattering {e[24] / ev:.3f}), list writes {e[25] / ev:.3f}")
    if e[18]:
        print(f"    takes: {e[18]:.3e}, of which with dynamic grabs {e[17]:.3e} ({e[19]:.3e} atomics); cycles per take "
              f"{e[9] / e[18]:.0f}, per take with grabs {e[16] / max(e[17], 1):.0f}, per take without "
              f"{(e[9] - e[16]) / max(e[18] - e[17], 1):.0f}")
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
g.close()

"""Lane occupancy of k_trace (needs the -DARTES_DEBUG_LANES build via ARTES_LIB_PATH).
usage: python tools/lane_stats.py [packets] [ENV=VAL,ENV=VAL ...]  (one variant per argument)
LS_WORKLOAD=cloudy: the configs[3] cloudy atmosphere (synthetic.make_cloudy, 0.45 micron, the
`phase` mode's 1-pixel detector at 0 degrees) instead of ray3d.
Since round 4 an iteration runs several steps ("Several steps per iteration"):
the per-iteration stop / move / retry counters then describe the iteration's last step only
(wave-steps, lanes and refills stay per iteration)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 5 * 10**7
variants = [dict(kv.split("=", 1) for kv in v.split(",")) if v else {} for v in (sys.argv[2:] or [""])]
cfg = driver.default_config()
for name in (os.environ.get("LS_WORKLOAD", "ray3d"),):
    if name == "cloudy":
        import tempfile

        atm = synthetic.make_cloudy(os.path.join(tempfile.mkdtemp(), "cloudy"), wavelength=(0.45,))
        cfg.apply("detector:type", "phase")
    else:
        atm = synthetic.make_config(name, share_matrix=True)
    det = driver.detector_geometry(cfg, atm["radial"][-1])
    g = Grid(atm, 0)
    g.set_profiling(True)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _tuning
    _tuning.apply(g)
    p = driver.run_params(cfg, det, 0, det_phi=1e-5 if name == "cloudy" else None, cell_depth=g.cell_depth(0),
                          packet_moments=False)
    for env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        g.run(p, 0, 10**5, 1)
        g.kernel_times()
        r = g.run(p, 0, n, 2024)
        kt = g.kernel_times()
        steps, lanes, refills = int(r.err[0]), int(r.err[30]), int(r.err[32])
        tsteps, tlanes = int(r.err[40]), int(r.err[41])
        C = r.counter("crossings")
        anystop, anyhit, nstop, nmove = int(r.err[48]), int(r.err[12]), int(r.err[1]), int(r.err[2])
        nretry, nsetup = int(r.err[4]), int(r.err[5])
        firuns, filanes, reflanes = int(r.err[6]), int(r.err[7]), int(r.err[8])
        hruns, hlanes = int(r.err[9]), int(r.err[10])
        f12, anyf12 = int(r.err[17]), int(r.err[22])
        f2, anyf2 = int(r.err[23]), int(r.err[24])
        print(f"{name} {env}: {g.last_kernel_ms():.1f} ms ({n / g.last_kernel_ms() / 1e3:.1f} Mpkt/s) trace {kt['trace'][0]:.1f} ms, "
              f"wave-steps {steps:.3e}, lanes/step {lanes / steps:.1f}, crossings/wave-step {C / steps:.1f}, "
              f"steps/refill {steps / max(refills, 1):.1f}, tail steps {tsteps / steps:.3f} at {tlanes / max(tsteps, 1):.1f} lanes, "
              f"iterations with a trace end {anystop / steps:.3f} (lanes {nstop / max(anystop, 1):.2f}), with an interaction {anyhit / steps:.3f}, "
              f"moving lanes/iteration {nmove / steps:.1f}, other-face retries {nretry / steps:.2f}, evaluations without a step {nsetup / steps:.2f}, "
              f"first-interaction block in {firuns / steps:.3f} of iterations ({filanes / max(firuns, 1):.2f} lanes), "
              f"lanes refilled per refill {reflanes / max(refills, 1):.1f}, "
              f"interaction block in {hruns / steps:.3f} of iterations ({hlanes / max(hruns, 1):.2f} lanes), "
              f"theta / phi evaluations {f12 / steps:.2f} lanes per wave-step, in {anyf12 / steps:.3f} of iterations "
              f"(phi: {f2 / steps:.2f} lanes, in {anyf2 / steps:.3f})",
              flush=True)
        rs = max(int(r.err[49]), 1)
        print(f"  per step of an iteration (of 64 lanes): idle {r.err[50] / rs:.2f}, parked {r.err[51] / rs:.2f}, "
              f"ended earlier in the iteration {r.err[52] / rs:.2f}, stepping {r.err[53] / rs:.2f}, "
              f"evaluating without a step {r.err[54] / rs:.2f}; crossings per step {C / rs:.2f}", flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    g.close()

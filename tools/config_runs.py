"""Throughput of BASELINE configs[3] and configs[4] at their stated shape on one GPU
(development tool; writes JSON for profiles/).

configs[3]: gas + Mie-cloud 3D grid (synthetic.make_cloudy: 16 x 6 x 6 cells, 25+ distinct
            matrices per wavelength), 50 wavelengths 0.45-0.95 micron.
            phase:    the reference's `phase` mode, 73 detector azimuths at wavelengths(1)
                      (ARTES.f90:206-250), 1-pixel detector, --packets per angle;
            spectrum: one call per wavelength (ARTES.f90:132-166), 1-pixel detector.
configs[4]: self-luminous gas with P-T dependent molecular opacities, 100 wavelengths
            (synthetic.make_self_luminous from tests/golden/molecular), planet source,
            `spectrum` mode, --packets per wavelength.
Every call is one artes_run of the drop-in's production parameters (packet moments off);
per call: wall time, packets/s, and the per-kernel HIP-event times.

usage: python tools/config_runs.py <out_dir> [--packets 1e8] [--which 3,4] [--phases K] [--lambdas K]
(--phases / --lambdas K: only K of the 73 angles / 50 wavelengths, evenly spaced -- the
short runs the rocprofv3 counter passes profile)
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tuning  # noqa: E402
from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402


def calls(grid, cfg, atm, items, n, seed, planet=False):
    """items: list of (label, wl index, det_phi) -> per-call records"""
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    out = []
    grid.set_profiling(True)
    for k, (label, wl, phi) in enumerate(items):
        cd = -1 if planet else grid.cell_depth(wl)
        p = driver.run_params(cfg, det, wl, det_phi=phi, cell_depth=cd, packet_moments=False)
        grid.kernel_times()
        t0 = time.perf_counter()
        res = grid.run(p, k * n, n, seed)
        dt = time.perf_counter() - t0
        kt = grid.kernel_times()
        c = res.counters.astype(np.float64)
        out.append({"call": label, "packets": n, "seconds": round(dt, 4), "mpackets_per_s": round(n / dt / 1e6, 2),
                    "crossings_per_packet": round(c[0] / n, 3), "scatters_per_packet": round(c[1] / n, 4),
                    "peels_per_packet": round(c[2] / n, 4),
                    "kernel_ms": {k2: round(v[0], 3) for k2, v in kt.items() if v[1]},
                    "k_event_ns_per_scatter": round(kt["event"][0] * 1e6 / max(c[1], 1.0), 4),
                    "errors": {str(i): int(e) for i, e in enumerate(res.err) if e}})
        print(json.dumps(out[-1]), flush=True)
    grid.set_profiling(False)
    return out


def summary(rows, what):
    n = sum(r["packets"] for r in rows)
    t = sum(r["seconds"] for r in rows)
    rates = [r["mpackets_per_s"] for r in rows]
    return {"what": what, "calls": len(rows), "packets": n, "seconds": round(t, 3),
            "mpackets_per_s": round(n / t / 1e6, 2), "min_call_mpackets_per_s": min(rates),
            "max_call_mpackets_per_s": max(rates)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--packets", type=float, default=1e8)
    ap.add_argument("--which", default="3,4")
    ap.add_argument("--seed", type=int, default=20171015)
    ap.add_argument("--phases", type=int, default=0, help="run only this many of the 73 phase angles")
    ap.add_argument("--lambdas", type=int, default=0, help="run only this many of the 50 wavelengths")
    a = ap.parse_args()
    n = int(a.packets)
    os.makedirs(a.out, exist_ok=True)
    tmp = tempfile.mkdtemp()
    which = set(a.which.split(","))
    if "3" in which:
        wl = tuple(np.round(np.linspace(0.45, 0.95, 50), 6))
        atm = synthetic.make_cloudy(os.path.join(tmp, "input", "cloudy50"), wavelength=wl)
        grid = Grid(atm, device=0)
        _tuning.apply(grid)   # ARTES_* of the environment (artes_set_tuning)
        res = {"config": "BASELINE configs[3]: gas + Mie cloud, 16x6x6 (r,theta,phi), 50 wavelengths 0.45-0.95 um, "
                         "star source, 1-pixel detector",
               "distinct_matrices": grid.num_matrices(), "packets_per_call": n}
        cfg = driver.default_config()
        cfg.apply("detector:type", "phase")
        phases = [(f"phi={np.degrees(p):.1f}", 0, p) for p in driver.phase_angles()]
        if a.phases:
            phases = [phases[i] for i in np.linspace(0, len(phases) - 1, a.phases).round().astype(int)]
        res["phase"] = calls(grid, cfg, atm, phases, n, a.seed)
        res["phase_summary"] = summary(res["phase"], f"phase curve at wavelengths(1) = 0.45 um, {len(phases)} angles")
        cfg = driver.default_config()
        cfg.apply("detector:type", "spectrum")
        det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
        spec = [(f"lambda={w:.4f}", i, det.det_phi) for i, w in enumerate(wl)]
        if a.lambdas:
            spec = [spec[i] for i in np.linspace(0, len(spec) - 1, a.lambdas).round().astype(int)]
        res["spectrum"] = calls(grid, cfg, atm, spec, n, a.seed + 1)
        res["spectrum_summary"] = summary(res["spectrum"], f"spectrum over {len(spec)} wavelengths")
        grid.close()
        json.dump(res, open(os.path.join(a.out, "configs3_cloudy.json"), "w"), indent=1)
        print(json.dumps({k: v for k, v in res.items() if "summary" in k}), flush=True)
    if "4" in which:
        fx = os.path.join(ROOT, "tests", "golden", "molecular", "self_luminous_100wl.npz")
        atm = synthetic.make_self_luminous(os.path.join(tmp, "input", "sl"), fx)
        grid = Grid(atm, device=0)
        _tuning.apply(grid)   # ARTES_* of the environment (artes_set_tuning)
        cfg = driver.default_config()
        cfg.apply("photon:source", "planet")
        cfg.apply("detector:type", "spectrum")
        det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
        items = [(f"lambda={w:.4f}", i, det.det_phi) for i, w in enumerate(atm["wavelength"])]
        res = {"config": "BASELINE configs[4]: self-luminous gas, molecular opacities (opacityMolecules), "
                         "19x6x4 (r,theta,phi), 100 wavelengths 1.0-2.7 um, planet source, spectrum mode",
               "packets_per_call": n}
        res["spectrum"] = calls(grid, cfg, atm, items, n, a.seed + 2, planet=True)
        res["spectrum_summary"] = summary(res["spectrum"], "thermal spectrum over 100 wavelengths")
        grid.close()
        json.dump(res, open(os.path.join(a.out, "configs4_thermal.json"), "w"), indent=1)
        print(json.dumps(res["spectrum_summary"]), flush=True)


if __name__ == "__main__":
    main()

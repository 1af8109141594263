"""Every k_event instantiation the engine's dispatch can pick (transport.hip, run_event_engine:
`ev_v` 1-18) against the CPU oracle, trajectory by trajectory.

The dispatch chooses from the call's shape: the scattering tables in LDS when the call's
matrices fit (LDS_T; a uniform atmosphere's one matrix) or only their cumulative part
(LDS_C; the cloudy atmosphere's ~9 matrices per wavelength), the detector in LDS (LDS_D;
25 x 25 imaging) or per-lane one-pixel sums (PIX1; `phase` / `spectrum`), 768- or 256-thread
blocks.  Each case forces one branch through the grid and the schedule tuning
(artes_set_tuning), asserts the instantiation that actually ran (artes_last_launch), and
compares 20k packets' records with the oracle's (ARTES.f90:4765-4984 peel-off, 819-846
scattering): >= 99.9 % of the packets with <= 20 scatterings identical to 1e-9, >= 99 %
overall, as tests/test_gpu_parity.py.  Two cases also read the 16-element matrix form
(tuning msym = 0) instead of the block-diagonal 4-element rows."""

import math

import numpy as np
import pytest

from artes_amd import driver, stats, synthetic

pytestmark = pytest.mark.gpu

# (variant, atmosphere, detector, tuning, expected k_event template arguments)
CASES = [
    (1, "uniform", "phase", {}, "1,0,1,768,0"),
    (2, "cloudy", "phase", dict(event_ldsu=0), "0,0,1,768,1"),
    (3, "cloudy", "imaging", dict(event_ldsu=0), "0,1,0,768,1"),
    (4, "cloudy", "imaging", dict(det_lds=0), "0,0,0,768,1"),
    (5, "cloudy", "phase", dict(event_ldsc=0, event_ldsu=0), "0,0,1,768,0"),
    (6, "uniform", "phase", dict(event_block=256), "1,0,1,256,0"),
    (7, "cloudy", "phase", dict(event_block=256), "0,0,1,256,0"),
    (8, "uniform", "imaging", {}, "1,1,0,768,0"),
    (9, "uniform", "imaging", dict(event_block=256), "1,1,0,256,0"),
    (10, "uniform", "imaging", dict(det_lds=0), "1,0,0,256,0"),
    (11, "cloudy", "imaging", dict(event_ldsc=0, event_ldsu=0), "0,1,0,768,0"),
    (12, "cloudy", "imaging", dict(event_block=256), "0,1,0,256,0"),
    (13, "cloudy", "imaging", dict(event_block=256, det_lds=0), "0,0,0,256,0"),
    (8, "uniform", "imaging", dict(msym=0), "1,1,0,768,0"),
    (3, "cloudy", "imaging", dict(msym=0), "0,1,0,768,1"),
    # round 6: the fixed-point detector (det_ordered, ORD) and the unpadded LDS tables (TPAD = 0)
    (14, "uniform", "imaging", dict(det_ordered=1), "1,0,0,768,0,2"),
    (15, "cloudy", "phase", dict(det_ordered=1), "0,0,0,768,1,2"),
    (16, "cloudy", "imaging", dict(det_ordered=1), "0,0,0,768,0,2"),
    (17, "cloudy", "phase", {}, "1,0,1,768,0,0,0"),
    (18, "cloudy", "imaging", {}, "1,1,0,768,0,0,0"),
    (19, "cloudy", "imaging40", dict(det_ordered=1), "0,0,0,768,1,1"),
    (20, "uniform", "imaging40", dict(det_ordered=1, event_ldsc=0), "0,0,0,768,0,1"),
]


@pytest.fixture(scope="module")
def atmospheres(tmp_path_factory):
    d = tmp_path_factory.mktemp("variants") / "input" / "cloudy"
    return {"uniform": synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8),
            "cloudy": synthetic.make_cloudy(str(d))}


@pytest.mark.parametrize("case", CASES, ids=[f"v{c[0]}-{c[1]}-{c[2]}-" + ("_".join(f"{k}{v}" for k, v in c[3].items())
                                                                          or "default") for c in CASES])
def test_event_variant_matches_oracle(require_gpu, oracle_mod, atmospheres, case):
    from artes_amd.engine import Grid

    variant, name, mode, tuning, targs = case
    atm = atmospheres[name]
    wl = 1 if name == "cloudy" else 0
    cfg = driver.default_config()
    if mode == "phase":
        cfg.apply("detector:type", "phase")
    if mode == "imaging40":   # (a detector whose fixed-point planes exceed LDS: ORD = 1)
        cfg.apply("detector:pixel", "40")
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    assert (det.nx == 1) == (mode == "phase")
    og = oracle_mod.OracleGrid(atm)
    grid = Grid(atm, device=0)
    grid.set_tuning(**tuning)
    p = driver.run_params(cfg, det, wl, det_phi=math.radians(60.0) if mode == "phase" else None,
                          cell_depth=og.cell_depth(wl))
    n = 20000
    seed = 900 + variant
    gpu = grid.trace(p, 0, n, seed)
    launched = grid.last_launch()
    grid.close()
    assert launched.endswith(f"k_event<{targs}>"), launched
    ref = og.run(p, 0, n, seed, records=True)[4]
    same = stats.records_agree(gpu, ref)
    short = ref[:, 1] <= 20
    assert same[short].mean() >= 0.999 and same.mean() >= 0.99, (variant, same.mean(), same[short].mean())
    assert gpu[:, 0].sum() > 0 and np.all(gpu[:, 1] >= 0)

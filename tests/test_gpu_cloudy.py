"""BASELINE configs[3]'s input shape on the GPU: a gas atmosphere with a Mie cloud patch
over several wavelengths, built through the restated setup path
(``artes_amd.synthetic.make_cloudy`` -> ``atmosphere.build``).

What this adds to tests/test_gpu_parity.py (uniform atmospheres, one matrix):
* per-cell extinction, albedo and scattering-matrix ids that vary from cell to cell,
  with more distinct matrices than k_event can stage in LDS (the matrix-id path);
* wavelength indices > 0 of a multi-wavelength grid;
* the multi-wavelength (``spectrum``) and multi-angle (``phase``) drivers of the CLI
  (``ARTES.f90:132-265``, ``write_output`` 3521-3621) on the GPU engine against the same
  CLI on the CPU oracle, same seeds.

Tolerance: per-packet histories as in test_gpu_parity (>= 99.9 % of packets with <= 20
scatterings identical to 1e-9, >= 99 % overall); the CLI outputs, being sums over the
same packets, to 1e-3 relative (a rare packet whose last-ulp history differs moves a sum
by far less than that)."""

import math

import numpy as np
import pytest

from artes_amd import atmosphere, driver, runner, stats, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cloudy(tmp_path_factory):
    root = tmp_path_factory.mktemp("cloudy")
    d = root / "input" / "cloudy"
    atm = synthetic.make_cloudy(str(d))
    return root, d, atm


def _same(gpu, ref):
    return stats.records_agree(gpu, ref)


@pytest.mark.parametrize("wl", [0, 1, 2])
def test_cloudy_trajectories_match_oracle(require_gpu, oracle_mod, cloudy, wl):
    from artes_amd.engine import Grid

    _, _, atm = cloudy
    grid = Grid(atm, device=0)
    assert grid.num_matrices() >= 20          # beyond k_event's LDS budget: per-cell matrix ids
    og = oracle_mod.OracleGrid(atm)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    p = driver.run_params(cfg, det, wl, cell_depth=og.cell_depth(wl))
    n = 20000
    gpu = grid.trace(p, 0, n, 2718 + wl)
    ref = og.run(p, 0, n, 2718 + wl, records=True)[4]
    grid.close()
    same = _same(gpu, ref)
    short = ref[:, 1] <= 20
    assert same[short].mean() >= 0.999 and same.mean() >= 0.99, (wl, same.mean(), same[short].mean())
    assert gpu[:, 1].mean() > 2.0              # several scatterings per packet in the cloud
    # the Mie matrix has P34 != 0, so multiple scattering turns U into V: the per-packet
    # comparison of V (records_agree) is not a comparison of zeros (~1/3 of the packets)
    assert (np.abs(ref[:, 6]) > 1e-6 * np.abs(ref[:, 0])).mean() > 0.1


@pytest.mark.parametrize("knob", [("det_lds", 0), ("event_block", 256)])
def test_cloudy_detector_lds_knob(require_gpu, cloudy, knob):
    """Detector accumulation in LDS or straight to HBM, and the LDS-detector k_event with L2
    tables (401 matrices) in 768- or 256-thread blocks: same packets, same image."""
    from artes_amd.engine import Grid

    _, _, atm = cloudy
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    grid = Grid(atm, device=0)
    p = driver.run_params(cfg, det, 1, cell_depth=grid.cell_depth(1))
    a = grid.run(p, 0, 200000, 5)
    la = grid.last_launch()
    grid.set_tuning(**{knob[0]: knob[1]})
    b = grid.run(p, 0, 200000, 5)
    assert grid.last_launch() != la
    grid.close()
    np.testing.assert_allclose(b.det, a.det, rtol=1e-9, atol=1e-300)
    assert np.array_equal(b.counters, a.counters)


@pytest.mark.parametrize("source,knob", [("star", ("pix1", 0)), ("planet", ("pix1", 0)), ("star", ("event_block", 256))])
def test_one_pixel_lane_sums_knob(require_gpu, cloudy, source, knob):
    """A one-pixel detector (spectrum / phase) keeps per-lane peel sums (LDS slots) reduced
    over the wave (k_event PIX1) instead of same-address atomics, in 768- or 256-thread
    blocks: same packets, same sums (to the summation order), counts exact; the planet
    source covers the I-only thermal peels."""
    from artes_amd.engine import Grid

    _, _, atm = cloudy
    if source == "planet":
        atm = synthetic.make_thermal(nr=10, ntheta=6, nphi=8, tau_abs=1.0, tau_sca=2.0, temperature=1100.0)
    cfg = driver.default_config()
    cfg.apply("detector:type", "phase")
    cfg.apply("photon:source", source)
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    assert det.nx == 1 and det.ny == 1
    grid = Grid(atm, device=0)
    p = driver.run_params(cfg, det, 0, det_phi=math.radians(40.0), cell_depth=-1 if source == "planet" else grid.cell_depth(0))
    a = grid.run(p, 0, 300000, 5)
    la = grid.last_launch()
    grid.set_tuning(**{knob[0]: knob[1]})
    b = grid.run(p, 0, 300000, 5)
    assert grid.last_launch() != la
    grid.close()
    np.testing.assert_allclose(a.det[:2], b.det[:2], rtol=1e-9, atol=1e-300)
    np.testing.assert_array_equal(a.det[2], b.det[2])
    assert np.array_equal(a.counters, b.counters) and a.det[0, 0].sum() > 0


ARTES_IN = """photon:source=star
photon:fstop=1d-5
photon:minimum=1d-20
star:temperature=5800
star:radius=1
planet:orbit=5
detector:type={mode}
detector:theta=90
detector:phi=90
detector:pixel=25
detector:distance=10
"""


def _rows(path):
    return np.array([[float(v) for v in l.split()] for l in open(path).read().splitlines()
                     if l.strip() and "#" not in l])


@pytest.mark.parametrize("mode,out", [("spectrum", "spectrum.dat"), ("phase", "phase.dat")])
def test_cloudy_cli_gpu_matches_oracle_cli(require_gpu, cloudy, mode, out):
    from test_cli import OracleTransport

    root, d, _ = cloudy
    (d / "artes.in").write_text(ARTES_IN.format(mode=mode))
    n = "4e4" if mode == "spectrum" else "5e3"
    assert runner.run(["cloudy", n, "-o", f"g_{mode}", "--seed", "11"], root=str(root)) == 0
    assert runner.run(["cloudy", n, "-o", f"o_{mode}", "--seed", "11"], root=str(root),
                      transport_factory=OracleTransport) == 0
    g = _rows(root / f"output/g_{mode}/output/{out}")
    o = _rows(root / f"output/o_{mode}/output/{out}")
    assert g.shape == o.shape and g.shape[0] == (3 if mode == "spectrum" else len(driver.phase_angles()))
    np.testing.assert_allclose(g[:, 0], o[:, 0])                       # wavelength / phase angle
    scale = np.abs(o[:, 1]).max()
    np.testing.assert_allclose(g[:, 1:], o[:, 1:], rtol=1e-3, atol=1e-3 * scale)
    assert np.all(o[:, 1] >= 0) and o[:, 1].max() > 0
    assert (root / f"output/g_{mode}/error.log").read_text() == ""
    if mode == "spectrum":   # optical_depth.dat (ARTES.f90:2457-2491): the same file from both runs
        od = (root / f"output/g_{mode}/output/optical_depth.dat").read_text()
        assert od == (root / f"output/o_{mode}/output/optical_depth.dat").read_text() and len(od.splitlines()) == 5


# ------------------------------------------------------------------------------------------
# configs[3] at its stated wavelength count: the same gas + Mie-cloud atmosphere over 50
# wavelengths 0.45-0.95 micron (401 distinct matrices; the k_event LDS_C path, the call's
# wavelength's ~9 matrices renumbered per call).  Trajectories at 8 of the 50 wavelengths and
# the full 50-wavelength spectrum through the CLI, GPU against oracle.

@pytest.fixture(scope="module")
def cloudy50(tmp_path_factory):
    root = tmp_path_factory.mktemp("cloudy50")
    d = root / "input" / "cloudy50"
    wl = tuple(np.round(np.linspace(0.45, 0.95, 50), 6))
    atm = synthetic.make_cloudy(str(d), wavelength=wl)
    return root, d, atm


@pytest.mark.parametrize("wl", [0, 7, 14, 21, 28, 35, 42, 49])
def test_cloudy50_trajectories_match_oracle(require_gpu, oracle_mod, cloudy50, wl):
    from artes_amd.engine import Grid

    _, _, atm = cloudy50
    grid = Grid(atm, device=0)
    assert grid.num_matrices() > 300
    og = oracle_mod.OracleGrid(atm)
    cfg = driver.default_config()
    cfg.apply("detector:type", "phase")
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    p = driver.run_params(cfg, det, wl, det_phi=math.radians(2.5 * wl), cell_depth=og.cell_depth(wl))
    n = 20000
    gpu = grid.trace(p, 0, n, 4242 + wl)
    ref = og.run(p, 0, n, 4242 + wl, records=True)[4]
    grid.close()
    same = _same(gpu, ref)
    short = ref[:, 1] <= 20
    assert same[short].mean() >= 0.999 and same.mean() >= 0.99, (wl, same.mean(), same[short].mean())
    assert gpu[:, 1].mean() > 1.0 and gpu[:, 0].sum() > 0


def test_cloudy50_spectrum_cli_gpu_matches_oracle_cli(require_gpu, cloudy50):
    from test_cli import OracleTransport

    root, d, _ = cloudy50
    (d / "artes.in").write_text(ARTES_IN.format(mode="spectrum"))
    assert runner.run(["cloudy50", "3000", "-o", "g50", "--seed", "12"], root=str(root)) == 0
    assert runner.run(["cloudy50", "3000", "-o", "o50", "--seed", "12"], root=str(root),
                      transport_factory=OracleTransport) == 0
    for f in ("spectrum.dat", "optical_depth.dat", "normalization.dat", "cell_depth.dat"):
        g = _rows(root / f"output/g50/output/{f}")
        o = _rows(root / f"output/o50/output/{f}")
        assert g.shape == o.shape and g.shape[0] == 50, f
        np.testing.assert_allclose(g[:, 0], o[:, 0], rtol=1e-12)
        scale = np.abs(o[:, 1:]).max(axis=0)
        assert np.all(np.abs(g[:, 1:] - o[:, 1:]) <= 1e-3 * scale + 1e-3 * np.abs(o[:, 1:])), f
    assert (root / "output/g50/error.log").read_text() == (root / "output/o50/error.log").read_text()

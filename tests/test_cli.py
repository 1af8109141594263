"""End-to-end drop-in CLI: input/<atm>/{artes.in,atmosphere.fits} -> output/<run>/...

The CPU tests inject the oracle as the per-rank transport to exercise the host-side
plumbing (argv grammar, directory handling, output formats); the GPU test drives the
real engine."""

import os

import numpy as np
import pytest

from artes_amd import atmosphere, fitsio, runner, synthetic
from artes_amd.engine import RunResult

ARTES_IN = """======================================
* ARTES input parameters
photon:source=star
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


def _make_input(root, mode="imaging_mono", name="ray3d", **spec):
    d = root / "input" / "atm"
    d.mkdir(parents=True)
    (d / "artes.in").write_text(ARTES_IN.format(mode=mode))
    atm = synthetic.make_config(name, **spec)
    atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"), atm)
    return d


class OracleTransport:
    def __init__(self, atm, device, oblateness):
        from oracle.oracle import OracleGrid

        self.g = OracleGrid(atm, oblateness)

    def cell_depth(self, wl):
        return self.g.cell_depth(wl)

    def thermal(self, wl, thermal_weight, ring):
        return self.g.thermal(wl, thermal_weight, ring)

    def run(self, params, first, n, seed, flow_global=False, flow_latitudinal=False):
        if flow_global or flow_latitudinal:
            d, t, c, e, fg, ft = self.g.run_flow(params, first, n, seed, threads=4)
            return RunResult(d, t, c, e, fg if flow_global else None, ft if flow_latitudinal else None)
        d, t, c, e, _ = self.g.run(params, first, n, seed, threads=4)
        return RunResult(d, t, c, e)


def test_usage_and_missing_input(tmp_path, capsys):
    assert runner.run([], root=str(tmp_path)) == 0
    assert "How to run ARTES" in capsys.readouterr().out
    assert runner.run(["nope", "1000"], root=str(tmp_path)) == 0


def test_imaging_mono_outputs_cpu_plumbing(tmp_path):
    _make_input(tmp_path, nr=6, ntheta=4, nphi=4)
    rc = runner.run(["atm", "2e4", "-o", "run1", "-k", "photon:fstop=2d-5", "--seed", "5"], root=str(tmp_path),
                    transport_factory=OracleTransport)
    assert rc == 0
    out = tmp_path / "output" / "run1"
    for f in ("error.log", "plot.dat", "input/artes.in", "input/atmosphere.fits", "output/stokes.fits",
              "output/error.fits", "output/photometry.dat", "output/normalization.dat", "output/cell_depth.dat"):
        assert (out / f).exists(), f
    assert (out / "input" / "artes.in").read_text().rstrip().endswith("photon:fstop=2d-5")
    s = fitsio.read(out / "output" / "stokes.fits")[0].data
    assert s.shape == (4, 25, 25) and s[0].sum() > 0


def test_spectrum_and_phase_modes(tmp_path):
    _make_input(tmp_path, mode="spectrum", name="iso", wavelength=(0.5, 0.7, 0.9))
    assert runner.run(["atm", "5e3", "-o", "spec", "--seed", "1"], root=str(tmp_path), transport_factory=OracleTransport) == 0
    lines = [l for l in (tmp_path / "output/spec/output/spectrum.dat").read_text().splitlines() if l.strip() and "#" not in l]
    assert len(lines) == 3 and float(lines[1].split()[0]) == pytest.approx(0.7)
    import shutil

    shutil.rmtree(tmp_path / "input")
    _make_input(tmp_path, mode="phase", name="iso")
    assert runner.run(["atm", "2e3", "-o", "ph", "--seed", "1"], root=str(tmp_path), transport_factory=OracleTransport) == 0
    rows = [l for l in (tmp_path / "output/ph/output/phase.dat").read_text().splitlines() if l.strip() and "#" not in l]
    assert len(rows) == 73 and float(rows[0].split()[0]) == 0.0 and float(rows[-1].split()[0]) == 180.0


def test_imaging_broad_accumulates_and_scales_by_last_wavelength(tmp_path):
    """imaging_broad (ARTES.f90:168-204): the thread sums accumulate over the wavelengths
    (array_start only at wl_count == 1) and each call rescales them by the CURRENT
    wavelength's package energy (959-975), so stokes.fits = sum_lambda(raw sums) x E(last),
    sum w^2 x E(last)^2; normalization.dat has the last wavelength only."""
    from artes_amd import driver
    from oracle.oracle import OracleGrid

    wls = (0.5, 0.7, 0.9)
    _make_input(tmp_path, mode="imaging_broad", name="ray3d", nr=6, ntheta=4, nphi=4, wavelength=wls)
    n, seed = 6000, 21
    assert runner.run(["atm", str(n), "-o", "bb", "--seed", str(seed)], root=str(tmp_path),
                      transport_factory=OracleTransport) == 0
    out = tmp_path / "output" / "bb" / "output"
    stokes = fitsio.read(out / "stokes.fits")[0].data
    err = fitsio.read(out / "error.fits")[0].data
    assert not (out / "photometry.dat").exists() and not (out / "spectrum.dat").exists()
    norm = np.loadtxt(out / "normalization.dat", ndmin=2)
    assert norm.shape[0] == 1 and norm[0, 0] == pytest.approx(0.9)
    # the same packets by hand: call k transports the global ids [k n, (k+1) n)
    atm = atmosphere.read_atmosphere_fits(str(tmp_path / "input" / "atm" / "atmosphere.fits"))
    cfg = driver.default_config()
    rt = float(atm["radial"][-1])
    det = driver.detector_geometry(cfg, rt)
    g = OracleGrid(atm)
    acc = 0.0
    for k in range(len(wls)):
        p = driver.run_params(cfg, det, k, cell_depth=g.cell_depth(k), packet_moments=False)
        acc = acc + g.run(p, k * n, n, seed, threads=4)[0][:3]
    E = [driver.package_energy(cfg, w * 1e-6, rt, n, det.det_phi) for w in wls]
    assert len(set(E)) == 3                                  # the energies differ per wavelength
    np.testing.assert_allclose(stokes, acc[0] * E[-1] * 1e-6 / det.pixel_scale ** 2, rtol=1e-12, atol=0)
    want = driver.scale_detector(acc, E[-1])
    assert np.all(want[1] == acc[1] * E[-1] ** 2)
    np.testing.assert_allclose(err, driver.error_image(want), rtol=1e-12, atol=0)
    assert stokes[0].sum() > 0


@pytest.mark.gpu
def test_imaging_broad_gpu_matches_oracle_cli(tmp_path, require_gpu):
    """The same imaging_broad run on the HIP engine and on the oracle (same seeds): the
    images are sums over the same packets."""
    _make_input(tmp_path, mode="imaging_broad", name="ray3d", nr=8, ntheta=6, nphi=8, wavelength=(0.5, 0.7, 0.9))
    assert runner.run(["atm", "3e4", "-o", "g", "--seed", "8"], root=str(tmp_path)) == 0
    assert runner.run(["atm", "3e4", "-o", "o", "--seed", "8"], root=str(tmp_path), transport_factory=OracleTransport) == 0
    g = fitsio.read(tmp_path / "output/g/output/stokes.fits")[0].data
    o = fitsio.read(tmp_path / "output/o/output/stokes.fits")[0].data
    scale = np.abs(o[0]).max()
    np.testing.assert_allclose(g, o, rtol=1e-3, atol=1e-3 * scale)
    assert o[0].sum() > 0 and (tmp_path / "output/g/error.log").read_text() == ""


def _make_thermal_input(root, mode="imaging_mono"):
    d = root / "input" / "hot"
    d.mkdir(parents=True)
    (d / "artes.in").write_text(ARTES_IN.replace("photon:source=star", "photon:source=planet").format(mode=mode))
    atm = synthetic.make_thermal(nr=8, ntheta=4, nphi=4, tau_abs=2.0, tau_sca=1.0,
                                 temperature=lambda rc: 1100.0 - 3e-3 * (rc - rc[0]), wavelength=(5.0, 10.0))
    atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"), atm)
    return atm


def _luminosity_rows(path):
    return [[float(x) for x in l.split()] for l in open(path).read().splitlines() if l.strip() and "#" not in l]


def test_planet_source_outputs_cpu_plumbing(tmp_path):
    """photon:source=planet: luminosity.dat (emitted luminosity = sum of the cell luminosities
    within the Monte-Carlo error), cell_luminosity.fits, thermal cell_depth.dat."""
    from oracle.oracle import OracleGrid

    atm = _make_thermal_input(tmp_path)
    n = 40000
    assert runner.run(["hot", str(n), "-o", "th", "--seed", "2"], root=str(tmp_path), transport_factory=OracleTransport) == 0
    out = tmp_path / "output" / "th" / "output"
    for f in ("stokes.fits", "error.fits", "photometry.dat", "luminosity.dat", "cell_luminosity.fits", "cell_depth.dat"):
        assert (out / f).exists(), f
    assert not (out / "normalization.dat").exists()
    cd, total, lum = OracleGrid(atm).thermal(0, True, False)
    rows = _luminosity_rows(out / "luminosity.dat")
    assert len(rows) == 1 and rows[0][0] == pytest.approx(5.0e-6)
    assert rows[0][1] == pytest.approx(lum.sum() * 1e-6, rel=0.02)          # emitted [W micron-1]
    assert 0.0 < rows[0][2] < rows[0][1]                                     # emergent < emitted
    np.testing.assert_allclose(fitsio.read(out / "cell_luminosity.fits")[0].data, lum, rtol=1e-12)
    assert int(open(out / "cell_depth.dat").read().split()[-1]) == cd
    s = fitsio.read(out / "stokes.fits")[0].data
    assert s[0].sum() > 0


@pytest.mark.gpu
def test_planet_source_cli_on_gpu(tmp_path, require_gpu):
    _make_thermal_input(tmp_path, mode="spectrum")
    assert runner.run(["hot", "2e5", "-o", "ths", "--seed", "4"], root=str(tmp_path)) == 0
    rows = _luminosity_rows(tmp_path / "output/ths/output/luminosity.dat")
    assert len(rows) == 2 and all(0.0 < r[2] < r[1] for r in rows)
    spec = [l for l in (tmp_path / "output/ths/output/spectrum.dat").read_text().splitlines() if l.strip() and "#" not in l]
    assert len(spec) == 2 and all(float(l.split()[1]) > 0 for l in spec)


@pytest.mark.gpu
def test_cli_on_gpu(tmp_path, require_gpu):
    _make_input(tmp_path, share_matrix=False)
    assert runner.run(["atm", "1e7", "-o", "gpu", "--seed", "3"], root=str(tmp_path)) == 0
    ph = open(tmp_path / "output/gpu/output/photometry.dat").read()
    from artes_amd.stats import read_photometry

    v = read_photometry(str(tmp_path / "output/gpu/output/photometry.dat"))
    assert v[1] == pytest.approx(2.503e-19, rel=0.01) and v[3] < 0
    assert os.path.getsize(tmp_path / "output/gpu/error.log") == 0

import math
import os

import numpy as np
import pytest

from artes_amd import driver, fitsio
from artes_amd.config import PC, PI, RunConfig


def test_detector_geometry_imaging():
    cfg = driver.default_config()
    d = driver.detector_geometry(cfg, 70011e3)
    assert (d.nx, d.ny) == (25, 25)
    assert d.x_max == pytest.approx(1.3 * 70011e3)
    assert d.det_theta == pytest.approx(PI / 2) and d.det_phi == pytest.approx(PI / 2)
    # plot.dat of the reference runs: fov=1.2167693E-01 mas (ARTES.f90:483)
    assert d.x_fov == pytest.approx(1.2167693e-01, rel=1e-7)
    assert d.pixel_scale == pytest.approx(d.x_fov / 25)


def test_detector_geometry_modes_and_clamps():
    cfg = RunConfig()
    cfg.apply("detector:type", "spectrum")
    cfg.apply("detector:phi", "0")
    d = driver.detector_geometry(cfg, 7e7)
    assert (d.nx, d.ny) == (1, 1) and d.det_phi == 1e-3           # ARTES.f90:492
    cfg2 = RunConfig()
    cfg2.apply("detector:type", "phase")
    d2 = driver.detector_geometry(cfg2, 7e7)
    assert d2.det_theta == pytest.approx(PI / 2) and (d2.nx, d2.ny) == (1, 1)
    cfg3 = RunConfig()
    cfg3.apply("detector:phi", "180")
    assert driver.detector_geometry(cfg3, 7e7).det_phi == pytest.approx(PI - 1e-3)


def test_phase_angles():
    a = driver.phase_angles()
    assert len(a) == 73
    assert a[0] == pytest.approx(1e-5 * PI / 180) and a[1] == pytest.approx(2.5 * PI / 180)
    assert a[-1] == pytest.approx((180 - 1e-5) * PI / 180)
    assert np.allclose(np.diff(a[1:-1]), 2.5 * PI / 180)


def test_package_energy_and_far_phase():
    cfg = driver.default_config()
    e = driver.package_energy(cfg, 0.7e-6, 70011e3, 10**6, PI / 2)
    flux = driver.planck(5800.0, 0.7e-6, 1)
    assert e == pytest.approx(PI * flux * 70011e3 ** 2 * cfg.r_star ** 2 / (cfg.orbit ** 2 * (10 * PC) ** 2 * 1e6))
    cfg.apply("detector:type", "phase")
    assert driver.package_energy(cfg, 0.7e-6, 70011e3, 10**6, 175 * PI / 180) == pytest.approx(0.19 * e)


def test_photometry_and_error_formulas():
    rng = np.random.default_rng(3)
    det = np.zeros((3, 4, 3, 3))
    det[0] = rng.normal(size=(4, 3, 3))
    det[0, 0] = np.abs(det[0, 0]) + 1
    det[2] = 5.0
    det[1] = det[0] ** 2 / 5.0 + 0.1
    ph = driver.photometry(det)
    assert ph[0] == pytest.approx(det[0, 0].sum())
    n = det[2, 0].sum()
    assert ph[1] == pytest.approx(math.sqrt(det[1, 0].sum() / n - (det[0, 0].sum() / n) ** 2) * math.sqrt(n))
    assert ph[8] == pytest.approx(math.hypot(det[0, 1].sum(), det[0, 2].sum()))
    err = driver.error_image(det)
    assert err.shape == (5, 3, 3)
    assert err[0, 1, 1] == pytest.approx(math.sqrt(det[1, 0, 1, 1] / 5 - (det[0, 0, 1, 1] / 5) ** 2) * math.sqrt(5))


def test_output_writers(tmp_path):
    det = np.zeros((3, 4, 25, 25))
    det[0, 0, 12, 12] = 2.0
    det[1, 0, 12, 12] = 4.0
    det[2, :, 12, 12] = 1.0
    driver.write_stokes_outputs(str(tmp_path), det, 0.5)
    s = fitsio.read(tmp_path / "stokes.fits")[0].data
    assert s.shape == (4, 25, 25) and s[0, 12, 12] == pytest.approx(2.0e-6 / 0.25)
    assert fitsio.read(tmp_path / "error.fits")[0].data.shape == (5, 25, 25)
    driver.write_photometry(str(tmp_path), 0.7e-6, driver.photometry(det))
    from artes_amd.stats import read_photometry

    ph = read_photometry(str(tmp_path / "photometry.dat"))
    assert ph[0] == pytest.approx(0.7) and ph[1] == pytest.approx(2.0e-6) and ph.size == 9
    driver.write_cell_depth(str(tmp_path), 0.7e-6, 3)
    driver.write_cell_depth(str(tmp_path), 0.8e-6, 4)
    lines = open(tmp_path / "cell_depth.dat").read().strip().splitlines()
    assert lines[-1].split()[-1] == "4" and lines[-2].split()[-1] == "3"
    driver.write_error_log(str(tmp_path / "error.log"), [0] * 31 + [2])
    assert open(tmp_path / "error.log").read().count("error 031") == 2

import hashlib
import json
import math
import os

import numpy as np
import pytest

from artes_amd import atmosphere, fitsio, opacity, synthetic
from conftest import GOLDEN

ANG = np.array([(i + 0.5) * math.pi / 180.0 for i in range(180)])


def test_simps_avg_matches_historic_scipy_rule():
    # even sample count: average of (Simpson first + trapezoid last) and (trapezoid first + Simpson rest)
    assert opacity.simps_avg([0.0, 1.0, 4.0, 9.0], [0.0, 1.0, 2.0, 3.0]) == pytest.approx(55.0 / 6.0, rel=1e-15)
    # odd sample count: plain Simpson, exact for cubics
    x = np.linspace(0, 2, 5)
    assert opacity.simps_avg(x ** 3, x) == pytest.approx(4.0, rel=1e-14)


@pytest.mark.parametrize("kind", ["iso", "hg", "ray"])
def test_normalised_phase_function(kind):
    s = synthetic.scatter_matrix(kind)
    assert s.shape == (180, 16, 1)
    assert 2 * math.pi * opacity.simps_avg(s[:, 0, 0] * np.sin(ANG), ANG) == pytest.approx(1.0, rel=1e-13)
    assert np.all(s[:, 0, 0] > 0)
    assert np.all(np.abs(s[:, 1, 0]) <= s[:, 0, 0] * (1 + 1e-12))        # |P12| <= P11


def test_isotropic_norm_is_not_exactly_one():
    # the reference's simps renormalisation of 1/(4 pi) gives 0.99996, not 1
    _, raw = opacity.isotropic([0.7])
    norm = 2 * math.pi * opacity.simps_avg(raw[:, 0, 0] * np.sin(ANG), ANG)
    assert norm == pytest.approx(0.99996, abs=2e-5) and norm != 1.0


def test_rayleigh_matrix_structure():
    s = synthetic.scatter_matrix("ray")[:, :, 0]
    # bins straddling 90 deg: P12/P11 ~ -1 (full linear polarisation), P33 ~ 0
    r = (s[89, 1] + s[90, 1]) / (s[89, 0] + s[90, 0])
    assert r == pytest.approx(-1.0, abs=5e-4)   # bin-edge averaging: -0.99970
    np.testing.assert_array_equal(s[:, 4], s[:, 1])
    np.testing.assert_array_equal(s[:, 5], s[:, 0])
    assert np.all(s[:, [2, 3, 6, 7, 8, 9, 11, 12, 13, 14]] == 0)


def test_hg_forward_peak():
    s = synthetic.scatter_matrix("hg")[:, 0, 0]
    assert s[0] / s[179] > 100 and np.all(np.diff(s) < 0)


def test_synthetic_inputs_match_survey_reference_inputs():
    h = json.load(open(os.path.join(GOLDEN, "survey_input_hashes.json")))

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()[:16]

    for name in ("iso", "hg", "ray3d"):
        a = synthetic.make_config(name, normalizer="simpson", share_matrix=True)
        for k in ("radial", "theta", "phi", "wavelength", "scattering", "absorption", "temperature"):
            assert sha(a[k]) == h[name][k], (name, k)
        assert list(np.shape(a["scattermatrix"])) == h[name]["shape_scattermatrix"]
    iso = synthetic.make_config("iso", normalizer="simpson")
    assert sha(iso["scattermatrix"]) == h["iso"]["scattermatrix"]      # bitwise-identical inputs


def _write_case(tmp_path):
    d = tmp_path / "input" / "case"
    (d / "opacity").mkdir(parents=True)
    op_r, sc_r = opacity.rayleigh([0.7, 1.2])
    op_i, sc_i = opacity.isotropic([0.7, 1.2], absorption=0.5, scattering=1.0)
    opacity.write_opacity_fits(str(d / "opacity" / "ray.fits"), op_r, sc_r)
    opacity.write_opacity_fits(str(d / "opacity" / "iso.fits"), op_i, sc_i)
    (d / "atmosphere.in").write_text(
        "[grid]\nradius: 1.\nradial: 50, 100\ntheta: 60, 90, 120\nphi: 180\n\n"
        "[composition]\ngas: off\nfits01: ray.fits\nfits02: iso.fits\n"
        "opacity01: 1, 1e-3, 0, nr, 0, ntheta, 0, nphi\n"
        "opacity02: 2, 2e-4, 0, 1, 1, 3, 0, 1\n")
    return d


def test_atmosphere_builder(tmp_path):
    d = _write_case(tmp_path)
    atm = atmosphere.build(str(d))
    assert atm["radial"].tolist() == [69911e3, 69961e3, 70011e3]
    assert atm["theta"].tolist() == [0, 60, 90, 120, 180] and atm["phi"].tolist() == [0, 180]
    assert atm["scattering"].shape == (2, 2, 4, 2) and atm["scattermatrix"].shape == (180, 16, 2, 2, 4, 2)
    op_r, _ = opacity.read_opacity_fits(str(d / "opacity" / "ray.fits"))
    op_i, _ = opacity.read_opacity_fits(str(d / "opacity" / "iso.fits"))
    k1 = 1.0 * op_r[3, 0] / 10.0                          # 1e-3 g/cm3 = 1 kg/m3, cm2/g / 10 = m2/kg
    assert atm["scattering"][0, 1, 3, 1] == pytest.approx(k1)
    k2s, k2a = 0.2 * op_i[3, 0] / 10.0, 0.2 * op_i[2, 0] / 10.0
    # overlap cell: opacities add (atmosphere.py:368-369); the matrix is mixed by extinction
    # weight only where `density` is already > 0, and `density` is filled after the
    # composition loop (atmosphere.py:371-377), so without gas the last region's matrix wins
    assert atm["scattering"][0, 0, 1, 0] == pytest.approx(k1 + k2s)
    assert atm["absorption"][0, 0, 1, 0] == pytest.approx(k2a)
    _, s_r = opacity.read_opacity_fits(str(d / "opacity" / "ray.fits"))
    _, s_i = opacity.read_opacity_fits(str(d / "opacity" / "iso.fits"))
    np.testing.assert_array_equal(atm["scattermatrix"][:, :, 0, 0, 1, 0], s_i[:, :, 0])
    np.testing.assert_array_equal(atm["scattermatrix"][:, :, 0, 0, 0, 1], s_r[:, :, 0])
    # density bookkeeping quirk: indexed by species number (atmosphere.py:371-377)
    assert atm["density"][0, 1, 0] == pytest.approx(1.0 + 0.2)
    # written file: nine HDUs in the reference order, read back positionally
    back = atmosphere.read_atmosphere_fits(str(d / "atmosphere.fits"))
    for k in atmosphere.HDU_ORDER:
        np.testing.assert_array_equal(back[k], atm[k])
    assert len(fitsio.read(str(d / "atmosphere.fits"))) == 9


def test_opacity_files_renormalised_in_place(tmp_path):
    d = _write_case(tmp_path)
    atmosphere.build(str(d))
    _, s = opacity.read_opacity_fits(str(d / "opacity" / "iso.fits"))
    assert 2 * math.pi * opacity.simps_avg(s[:, 0, 1] * np.sin(ANG), ANG) == pytest.approx(1.0, rel=1e-13)

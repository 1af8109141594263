"""The oracle's thermal source (photon:source=planet) and Lambertian surface, pinned by
analytic known answers.

The reference's frozen runs (tests/golden/) cover the star source only, so parity of
these two paths with the reference itself is UNPINNED; what is pinned here is the
oracle's restatement of
  - grid_initialize(2), planet branch (ARTES.f90:2359-2453): cell_depth, cell volumes,
    Planck function, luminosity weights, total emissivity -- against an independent
    numpy evaluation;
  - emit_photon's cell sampling and weights (1117-1266, 599-607): the emitted-luminosity
    estimator is unbiased;
  - peel_thermal (4519-4598): the optically thin flux of an isothermal shell is the
    visible (un-eclipsed) fraction of its luminosity over 4 pi;
  - lambertian + peel_surface (1369-1402, 4600-4708): a Lambert sphere seen at 90
    degrees phase reflects (2/3) (R_s / R_top)^2 / pi^2 of the packets' weight.
"""

import math

import numpy as np
import pytest

from artes_amd import driver, synthetic


def _cfg(**kv):
    cfg = driver.default_config()
    for k, v in kv.items():
        cfg.apply(k.replace("__", ":"), v)
    return cfg


def _params(atm, cfg, cell_depth=-1):
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    return driver.run_params(cfg, det, 0, cell_depth=cell_depth)


def _numpy_thermal(atm, weight=True, ring=False):
    """Independent restatement of ARTES.f90:2274-2300, 2359-2453 (numpy, no shared code)."""
    hh, cc, kb = 6.62606957e-34, 2.99792458e8, 1.3806488e-23
    lam = float(atm["wavelength"][0]) * 1e-6
    r, th, ph = atm["radial"], np.radians(atm["theta"]), np.radians(atm["phi"])
    nr, nt, nph = r.size - 1, th.size - 1, ph.size
    ab = atm["absorption"][0]                                  # [nphi][ntheta][nr]
    t = atm["temperature"]
    dphi = np.diff(np.append(ph, 2 * np.pi)) if nph > 1 else np.array([2 * np.pi])
    vol = ((1 / 3) * (r[1:] ** 3 - r[:-1] ** 3)[None, None, :] * (np.cos(th[:-1]) - np.cos(th[1:]))[None, :, None]
           * dphi[:, None, None])
    start = 2 if ring else 0                                   # a ring skips the two outer cells
    tau = np.cumsum((ab * np.diff(r)[None, None, :])[:, :, ::-1][:, :, start:], axis=2)   # from the top down
    depth = []
    for k in range(nph):
        for j in range(nt):
            idx = np.nonzero(tau[k, j] > 5.0)[0]
            i = start + (idx[0] if idx.size else nr - 1 - start)
            depth.append(nr - i - 1)
    cd = min(depth)
    b = (2 * hh * cc * cc / lam ** 5) / np.expm1(hh * cc / (lam * kb * np.where(t > 0, t, 1.0)))
    on = np.zeros_like(t, dtype=bool)
    on[:, :, cd:] = (t[:, :, cd:] > 0) & (ab[:, :, cd:] > 0)
    norm = np.sum(np.where(on, ab * b * vol, 0.0))
    w = np.where(on, norm / np.where(on, vol * ab * b, 1.0), 0.0) if weight else on.astype(float)
    lum = np.where(on, 4 * np.pi * vol * ab * b, 0.0)
    return cd, float(np.sum(lum * w)), lum, w


@pytest.mark.parametrize("weight", [True, False])
@pytest.mark.parametrize("ring", [False, True])
def test_thermal_tables_match_independent_formulas(oracle_mod, weight, ring):
    lapse = lambda rc: 1500.0 - 5e-3 * (rc - rc[0])   # noqa: E731 -- K, decreasing outward
    atm = synthetic.make_thermal(nr=12, ntheta=6, nphi=4, tau_abs=8.0, tau_sca=1.0, temperature=lapse)
    cd, tot, lum = oracle_mod.OracleGrid(atm).thermal(0, weight, ring)
    cd_n, tot_n, lum_n, _ = _numpy_thermal(atm, weight, ring)
    assert cd == cd_n
    assert 0 < cd < 12
    assert tot == pytest.approx(tot_n, rel=1e-10)
    # (r1^3 - r0^3 of a thin shell cancels ~4 digits: numpy pow vs r*r*r differ at 1e-12)
    np.testing.assert_allclose(lum, lum_n, rtol=1e-10, atol=0)


@pytest.mark.parametrize("weight", ["on", "off"])
def test_emitted_luminosity_estimator_is_unbiased(oracle_mod, weight):
    """E[flux_emitted] * e_pack * N = sum of the cell luminosities (ARTES.f90:2439, 3677)."""
    lapse = lambda rc: 1200.0 - 4e-3 * (rc - rc[0])   # noqa: E731
    atm = synthetic.make_thermal(nr=10, ntheta=4, nphi=4, tau_abs=3.0, tau_sca=0.5, temperature=lapse)
    g = oracle_mod.OracleGrid(atm)
    cfg = _cfg(photon__source="planet", photon__weight=weight, detector__pixel="5")
    p = _params(atm, cfg)
    n = 200000
    det, tot, cnt, err, _ = g.run(p, 0, n, 7)
    cd, total, lum = g.thermal(0, weight == "on", False)
    est = tot[8] * total / n
    truth = lum.sum()
    if weight == "off":
        assert tot[8] == n                    # every packet carries weight 1
    # weights 1/cell_weight vary with temperature: a few per mille at 2e5 packets
    assert est == pytest.approx(truth, rel=1e-2)
    assert 0.0 < tot[9] < tot[8]              # some of the emitted weight escapes
    assert int(cnt[3]) == n


def _shadow_fraction(r0, r1):
    """Fraction of the shell r0 < r < r1 hidden from a distant observer by the sphere r0."""
    v_shadow = 2 * math.pi / 3 * (r1 ** 3 - (r1 * r1 - r0 * r0) ** 1.5 - r0 ** 3)
    return v_shadow / (4 * math.pi / 3 * (r1 ** 3 - r0 ** 3))


def test_thermal_peel_optically_thin_shell(oracle_mod):
    """peel_thermal of a transparent isothermal shell: each packet adds exp(-tau)/(4 pi)
    unless the planet eclipses it, so sum_I / N = (1 - shadow) / (4 pi)."""
    atm = synthetic.make_thermal(nr=8, ntheta=4, nphi=8, tau_abs=1e-9, tau_sca=0.0, temperature=800.0)
    g = oracle_mod.OracleGrid(atm)
    cfg = _cfg(photon__source="planet", photon__weight="off", photon__scattering="off", detector__pixel="9")
    p = _params(atm, cfg)
    n = 400000
    det, tot, cnt, err, _ = g.run(p, 0, n, 11)
    r0, r1 = float(atm["radial"][0]), float(atm["radial"][-1])
    want = (1.0 - _shadow_fraction(r0, r1)) / (4 * math.pi)
    got = det[0, 0].sum() / n
    # binomial error of the visible fraction
    q = 1 - _shadow_fraction(r0, r1)
    sig = math.sqrt(q * (1 - q) / n) / (4 * math.pi)
    assert abs(got - want) < 4 * sig
    assert det[0, 1:].sum() == 0.0                      # thermal peels carry I only
    assert det[2, 0].sum() == pytest.approx(det[0, 0].sum() * 4 * math.pi, rel=1e-6)   # one count per peel
    assert det[2, 1:].sum() == 0.0                      # counted for I alone (ARTES.f90:4581)


def test_lambert_surface_at_quadrature(oracle_mod):
    """Star light on a transparent atmosphere over a Lambert surface (albedo 1), detector at
    90 degrees phase: sum_I / N = (2/3) (R_s/R_top)^2 / pi^2 (integral of mu0 mu / pi over
    the lit and visible quarter of the sphere)."""
    atm = synthetic.make(kind="iso", nr=4, ntheta=1, nphi=1, tau=1e-9)
    g = oracle_mod.OracleGrid(atm)
    cfg = _cfg(planet__surface_albedo="1", detector__pixel="9")
    p = _params(atm, cfg)
    n = 400000
    det, tot, cnt, err, _ = g.run(p, 0, n, 5)
    rs, rt = float(atm["radial"][0]), float(atm["radial"][-1])
    want = (2.0 / 3.0) * (rs / rt) ** 2 / math.pi ** 2
    got = det[0, 0].sum() / n
    # per-packet weight in [0, 1/pi] on a hit fraction (rs/rt)^2
    sig = math.sqrt(((rs / rt) ** 2) / (math.pi ** 2 * 4) / n)
    assert abs(got - want) < 5 * sig
    assert got == pytest.approx(want, rel=0.02)
    assert det[0, 1:].sum() == 0.0
    assert int(err.sum()) == 0

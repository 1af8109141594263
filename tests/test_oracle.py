"""Pinning the CPU oracle (oracle/artes_oracle.c) before it is trusted as the checker.

(1) Frozen reference outputs (tests/golden/reference_runs, produced by the reference
    Fortran during the survey, see tests/golden/README.md): the oracle, driven with the
    same inputs, must agree in photometry and per-pixel Stokes images within the
    Monte-Carlo sigma (honest packet-level sigma for both sides, tests/golden/README.md).
(2) Analytic known answers: optically thin single scattering (intensity from the lit
    and visible shell volume; Rayleigh polarisation at 90 deg), isotropic Q=U=V=0,
    the reference's own normalization.dat numbers.
"""

import math
import os

import numpy as np
import pytest

from artes_amd import driver, stats, synthetic
from conftest import GOLDEN

REF = os.path.join(GOLDEN, "reference_runs")
SEED = 424242


def _setup(name, **over):
    atm = synthetic.make_config(name, normalizer="simpson", **over)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    return atm, cfg, det


def _run_oracle(oracle_mod, atm, cfg, det, n, seed=SEED, threads=8):
    g = oracle_mod.OracleGrid(atm)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    raw, tot, cnt, err, _ = g.run(p, 0, n, seed, threads=threads)
    return g, p, raw, tot, cnt, err


@pytest.mark.parametrize("name,run", [("iso", "t_iso_ARTES_det_1e6"), ("hg", "t_hg_ARTES_det_1e6"),
                                      ("ray3d", "t_ray3d_ARTES_det_1e6")])
def test_oracle_matches_reference_runs(oracle_mod, name, run):
    atm, cfg, det = _setup(name)
    n = 4 * 10**6             # 4x the reference run: a stable per-packet variance estimate
    _, _, raw, tot, cnt, err = _run_oracle(oracle_mod, atm, cfg, det, n)
    assert err.sum() == 0
    E = driver.package_energy(cfg, 0.7e-6, float(atm["radial"][-1]), n, det.det_phi)
    ph = driver.photometry(driver.scale_detector(raw[:3], E))
    ref = stats.load_reference_run(os.path.join(REF, run))
    rph = ref["photometry"]          # lambda, I, sI, Q, sQ, U, sU, V, sV (x1e-6)
    s_mine = stats.total_sigma_scaled(tot, n, E) * 1e-6
    s_ref = stats.total_sigma_scaled(tot, n, E, 10**6) * 1e-6
    for k, col in ((0, 1), (1, 3), (2, 5)):
        mine = ph[2 * k] * 1e-6
        comb = math.hypot(s_mine[k], s_ref[k])
        assert abs(mine - rph[col]) <= 4.0 * comb + 1e-12 * abs(rph[1]), (name, k, mine, rph[col], comb)
    assert ph[6] == 0.0 and rph[7] == 0.0                   # V
    cmp = stats.compare_to_reference(raw, n, E, det.pixel_scale, ref, 10**6)
    assert cmp["n_pixels"] > 100
    # per-pixel z-scores: N(0,1) has rms 1, median |z| 0.674
    # SURVEY.md §8(d) / BASELINE.md: RMS(z) <= 1.2 and |mean z| <= 0.1
    assert 0.8 < cmp["rms_z"] <= 1.2 and abs(cmp["mean_z"]) <= 0.1, cmp
    assert 0.5 < cmp["median_abs_z"] < 0.9 and cmp["frac_gt4"] <= 0.02, cmp
    # event statistics of the survey's counter-instrumented reference: C, S per packet
    C_ref = {"iso": 36.8, "hg": 108.0, "ray3d": 109.6}[name]
    assert cnt[0] / n == pytest.approx(C_ref, rel=0.01)
    assert cnt[1] / n == pytest.approx({"iso": 2.57, "hg": 2.50, "ray3d": 2.56}[name], abs=0.03)


def test_oracle_against_independent_reference_seeds(oracle_mod):
    """ray3d photometry vs four independent 1e6-packet reference runs (chi^2 over runs)."""
    atm, cfg, det = _setup("ray3d")
    n = 10**6
    _, _, raw, tot, _, _ = _run_oracle(oracle_mod, atm, cfg, det, n, seed=7)
    E = driver.package_energy(cfg, 0.7e-6, float(atm["radial"][-1]), n, det.det_phi)
    sig = stats.total_sigma_scaled(tot, n, E)[0] * 1e-6
    mine = raw[0, 0].sum() * E * 1e-6
    refs = [stats.load_reference_run(os.path.join(REF, r))["photometry"][1]
            for r in ("t_ray3d_ARTES_det_1e6", "ray2", "ray_ns1d", "ray_ns8")]
    # the four reference runs are independent; each differs from this run by both errors
    chi2 = sum(((x - mine) / (sig * math.sqrt(2))) ** 2 for x in refs)
    assert chi2 < 16.0, (chi2, refs, mine, sig)                         # 4 dof, p ~ 0.003


def test_isotropic_is_unpolarised(oracle_mod):
    atm, cfg, det = _setup("iso")
    _, _, raw, _, _, _ = _run_oracle(oracle_mod, atm, cfg, det, 20000)
    assert np.all(raw[0, 1:] == 0.0) and raw[0, 0].sum() > 0


def _lit_visible_volume(r_p: float, r_t: float) -> float:
    """Volume of the shell r_p<r<r_t that is both illuminated from +x and visible from +y.

    At radius r and n_z = mu, with s = sqrt(1-mu^2) and c = sqrt(1 - r_p^2/r^2), a point
    is lit iff n_x >= -c and visible iff n_y >= -c; the azimuthal measure of both is
    L = pi - 2 acos(a) + 2 asin(a) + max(0, 2 acos(a) - pi/2), a = c/s (L = 2 pi for a>=1)."""
    xg, wg = np.polynomial.legendre.leggauss(48)
    r = 0.5 * (r_t - r_p) * xg + 0.5 * (r_t + r_p)
    wr = 0.5 * (r_t - r_p) * wg
    m = 400000
    mu = (np.arange(m) + 0.5) / m * 2.0 - 1.0
    s = np.sqrt(1.0 - mu * mu)
    vol = 0.0
    for ri, wi in zip(r, wr):
        c = math.sqrt(max(0.0, 1.0 - (r_p / ri) ** 2))
        a = np.minimum(c / s, 1.0)
        L = math.pi - 2 * np.arccos(a) + 2 * np.arcsin(a) + np.maximum(0.0, 2 * np.arccos(a) - math.pi / 2)
        vol += wi * ri * ri * L.mean() * 2.0
    return vol


def test_thin_limit_single_scattering_intensity(oracle_mod):
    """tau = 1e-6: detector sum = N (1-fstop) kappa P11(90deg) V_lit,visible / (pi R_top^2)."""
    atm, cfg, det = _setup("iso", tau=1e-6)
    n = 400000
    _, _, raw, tot, cnt, _ = _run_oracle(oracle_mod, atm, cfg, det, n)
    rp, rt = float(atm["radial"][0]), float(atm["radial"][-1])
    kappa = 1e-6 / 100e3
    P = atm["scattermatrix"][:, 0, 0, 0, 0, 0]
    p90 = 0.5 * (P[89] + P[90])                 # interpolation between the 89.5 / 90.5 deg bins
    expect = n * (1 - cfg.fstop) * kappa * p90 * _lit_visible_volume(rp, rt) / (math.pi * rt * rt)
    got = raw[0, 0].sum()
    sig = stats.total_sigma_raw(tot, n)[0]
    assert abs(got - expect) < 4 * sig + 2e-4 * expect, (got, expect, sig)
    assert sig / expect < 5e-3


def test_thin_limit_rayleigh_polarisation(oracle_mod):
    """Single Rayleigh scattering at 90 deg is fully polarised: Q/I -> P12/P11(90) (stored as -Q)."""
    atm, cfg, det = _setup("ray1d", tau=1e-6)
    n = 200000
    _, _, raw, tot, _, _ = _run_oracle(oracle_mod, atm, cfg, det, n)
    P = atm["scattermatrix"][:, :, 0, 0, 0, 0]
    ratio = (P[89, 1] + P[90, 1]) / (P[89, 0] + P[90, 0])            # -0.9997
    I, Q, U = raw[0, 0].sum(), raw[0, 1].sum(), raw[0, 2].sum()
    assert Q / I == pytest.approx(ratio, abs=2e-4)
    assert abs(U / I) < 3e-3


def test_normalization_matches_reference_output(tmp_path):
    """planck_function / normalization.dat (ARTES.f90:3643-3648) vs the reference's own file."""
    cfg = driver.default_config()
    rt = 69911e3 + 100e3
    driver.write_normalization(str(tmp_path), cfg, 0.7e-6, rt)
    mine = np.loadtxt(tmp_path / "normalization.dat")
    ref = np.loadtxt(os.path.join(REF, "t_ray3d_ARTES_det_1e6", "normalization.dat"))
    np.testing.assert_allclose(mine, ref, rtol=1e-13)
    cd = open(os.path.join(REF, "t_ray3d_ARTES_det_1e6", "cell_depth.dat")).read().split()[-1]
    assert int(cd) == 0


def test_oracle_shard_and_thread_invariance(oracle_mod):
    atm, cfg, det = _setup("hg")
    g = oracle_mod.OracleGrid(atm)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    a = g.run(p, 0, 30000, 11, threads=8)
    b1 = g.run(p, 0, 12345, 11, threads=1)
    b2 = g.run(p, 12345, 30000 - 12345, 11, threads=3)
    np.testing.assert_allclose(a[0], b1[0] + b2[0], rtol=1e-10, atol=1e-300)
    np.testing.assert_array_equal(a[2], b1[2] + b2[2])

"""Known answers on the HIP engine itself (not through the oracle): the analytic pins of
tests/test_oracle.py, run through the C ABI, so the GPU path has a pin of its own.

* Optically thin single scattering (tau = 1e-6, isotropic): the detector sum is
  N (1 - fstop) kappa P11(90 deg) V_lit,visible / (pi R_top^2) -- one scattering at a
  point of the lit shell, peeled to the detector at 90 deg (ARTES.f90:660-685 forced
  first interaction, 4710-4990 peel-off), with the lit-and-visible shell volume in
  closed form (tests/test_oracle.py::_lit_visible_volume).
* Single Rayleigh scattering at 90 deg is fully polarised: Q/I = P12/P11(90 deg)
  (opacityRayleigh.py:98-104; the detector stores -Q, ARTES.f90:4956), U/I -> 0.
* Isotropic scattering never polarises: Q = U = V = 0 exactly.
Tolerance: 4 Monte-Carlo sigma (packet-level) plus the quadrature error of the volume.
"""

import math

import numpy as np
import pytest

from artes_amd import driver, stats, synthetic
from test_oracle import _lit_visible_volume

pytestmark = pytest.mark.gpu


def _run(name, n, seed, **over):
    from artes_amd.engine import Grid

    atm = synthetic.make_config(name, normalizer="simpson", **over)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    grid = Grid(atm, device=0)
    p = driver.run_params(cfg, det, 0, cell_depth=grid.cell_depth(0))
    res = grid.run(p, 0, n, seed)
    grid.close()
    return atm, cfg, res


def test_gpu_thin_limit_single_scattering_intensity(require_gpu):
    n = 4 * 10**6
    atm, cfg, res = _run("iso", n, 1234, tau=1e-6)
    rp, rt = float(atm["radial"][0]), float(atm["radial"][-1])
    kappa = 1e-6 / 100e3
    P = atm["scattermatrix"][:, 0, 0, 0, 0, 0]
    p90 = 0.5 * (P[89] + P[90])
    expect = n * (1 - cfg.fstop) * kappa * p90 * _lit_visible_volume(rp, rt) / (math.pi * rt * rt)
    got = res.det[0, 0].sum()
    sig = stats.total_sigma_raw(res.totals, n)[0]
    assert abs(got - expect) < 4 * sig + 2e-4 * expect, (got, expect, sig)
    assert sig / expect < 2e-3
    # one (forced) scattering per packet: roulette (fstop) and a second interaction are rare
    assert abs(res.counter("scatters") - n) <= 1e-3 * n
    assert np.all(res.det[0, 1:] == 0.0)


def test_gpu_thin_limit_rayleigh_polarisation(require_gpu):
    n = 2 * 10**6
    atm, cfg, res = _run("ray1d", n, 4321, tau=1e-6)
    P = atm["scattermatrix"][:, :, 0, 0, 0, 0]
    ratio = (P[89, 1] + P[90, 1]) / (P[89, 0] + P[90, 0])            # -0.9997
    I, Q, U, V = (res.det[0, k].sum() for k in range(4))
    assert Q / I == pytest.approx(ratio, abs=2e-4)
    assert abs(U / I) < 1e-3
    assert V == 0.0                                                   # Rayleigh: P34 = 0


def test_gpu_isotropic_is_unpolarised(require_gpu):
    _, _, res = _run("iso", 10**6, 99)
    assert res.det[0, 0].sum() > 0 and np.all(res.det[0, 1:] == 0.0)


# ------------------------------------------------------------------------------------------
# The drop-in's other drivers on the HIP path, pinned by analytic answers of their own
# ("What's missing" 2): the `phase` mode (ARTES.f90:206-250), the Lambertian
# surface (lambertian 1369-1402, peel_surface 4600-4708) and the planet source (emission
# 1117-1266, peel_thermal 4519-4598, photon_package 2535).  They run through the CLI
# (runner.run -> phase.dat / photometry.dat), with `transport_factory=None` the HIP engine.

PHASE_IN = """photon:source={source}
photon:fstop=1d-5
photon:minimum=1d-20
star:temperature=5800
star:radius=1
planet:orbit=5
planet:surface_albedo={albedo}
detector:type={mode}
detector:theta=90
detector:phi=90
detector:pixel=25
detector:distance=10
"""


def _cli(root, name, atm, n, seed, source="star", albedo="0", mode="phase", transport_factory=None):
    from artes_amd import atmosphere, runner

    d = root / "input" / name
    d.mkdir(parents=True, exist_ok=True)
    (d / "artes.in").write_text(PHASE_IN.format(source=source, albedo=albedo, mode=mode))
    atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"), atm)
    assert runner.run([name, str(int(n)), "-o", name, "--seed", str(seed)], root=str(root),
                      transport_factory=transport_factory) == 0
    assert (root / "output" / name / "error.log").read_text() == ""
    return root / "output" / name / "output"


def _phase_rows(path):
    return np.array([[float(v) for v in l.split()] for l in open(path).read().splitlines() if l.strip() and "#" not in l])


def lambert_phase(alpha):
    """Lambert phase function of a sphere, Phi(alpha) = [sin a + (pi - a) cos a] / pi."""
    return (np.sin(alpha) + (math.pi - alpha) * np.cos(alpha)) / math.pi


def check_lambert_phase_curve(tmp_path, n, transport_factory=None, grid_factory=None):
    """A Lambert sphere (surface albedo 1) under a transparent atmosphere (tau = 1e-9: the first
    optical depth trace reaches the surface with tau_first < 1e-6, so no forced interaction,
    ARTES.f90:666-671, and each packet reflects once, 764-772), seen at the 73 phase angles:
    phase.dat's Stokes I(alpha) = E N (2/3) (R_s / R_top)^2 Phi(alpha) / pi x 1e-6 (the
    integral of mu0 mu / pi over the lit and visible part of the sphere; E = package energy of
    a full-disk call, photon_package 2509-2539), within 4 packet-level sigma -- taken from the
    same packets rerun with the packet moments on (the CLI's sums are checked to be those)."""
    from artes_amd.config import PI

    atm = synthetic.make(kind="iso", nr=4, ntheta=1, nphi=1, tau=1e-9)
    seed = 31
    out = _cli(tmp_path, "lam", atm, n, seed, albedo="1", transport_factory=transport_factory)
    rows = _phase_rows(out / "phase.dat")
    assert rows.shape == (73, 9)
    angles = np.array(driver.phase_angles())
    np.testing.assert_allclose(rows[1:-1, 0], np.degrees(angles[1:-1]), rtol=1e-12)
    rs, rt = float(atm["radial"][0]), float(atm["radial"][-1])
    cfg = driver.default_config()
    cfg.apply("detector:type", "phase")
    cfg.apply("planet:surface_albedo", "1")
    e_full = driver.package_energy(cfg, 0.7e-6, rt, int(n), 0.0)
    want = e_full * n * (2.0 / 3.0) * (rs / rt) ** 2 * lambert_phase(angles) / math.pi * 1e-6
    g = grid_factory(atm)
    det = driver.detector_geometry(cfg, rt)
    for k, phi in enumerate(angles):
        p = driver.run_params(cfg, det, 0, det_phi=phi, cell_depth=g.cell_depth(0), packet_moments=True)
        res = g.run(p, k * int(n), int(n), seed)
        e_k = driver.package_energy(cfg, 0.7e-6, rt, int(n), phi)
        assert rows[k, 1] == pytest.approx(res.det[0, 0].sum() * e_k * 1e-6, rel=1e-12, abs=0)   # the CLI's packets
        sig = stats.total_sigma_raw(res.totals, int(n))[0] * e_k * 1e-6
        assert abs(rows[k, 1] - want[k]) <= 4.0 * sig + 1e-12 * want[0], (k, np.degrees(phi), rows[k, 1], want[k], sig)
        assert np.all(rows[k, 3::2] == 0.0)             # a Lambert surface depolarises: Q = U = V = 0
    assert rows[0, 1] > 0 and rows[-1, 1] < 1e-3 * rows[0, 1]
    return rows, want


def check_thin_rayleigh_phase_polarisation(tmp_path, n, transport_factory=None):
    """Optically thin Rayleigh atmosphere (tau = 1e-6) over a black planet, at the 73 phase
    angles: every peel is a single scattering at angle pi - alpha, so phase.dat's Q / I is the
    matrix ratio P12 / P11 there -- linearly interpolated between bin centres as scatter_photon
    does (ARTES.f90:1448-1530), the detector storing -Q (4956) -- and U / I -> 0."""
    atm = synthetic.make_config("ray1d", tau=1e-6, normalizer="simpson")
    out = _cli(tmp_path, "ray", atm, n, 77, transport_factory=transport_factory)
    rows = _phase_rows(out / "phase.dat")
    angles = np.array(driver.phase_angles())
    P = atm["scattermatrix"][:, :, 0, 0, 0, 0]
    centres = np.arange(180) + 0.5
    theta = 180.0 - np.degrees(angles)
    want = np.interp(theta, centres, P[:, 1]) / np.interp(theta, centres, P[:, 0])
    I, Q, U = rows[:, 1], rows[:, 3], rows[:, 5]
    assert np.all(I > 0)
    np.testing.assert_allclose(Q / I, want, rtol=0, atol=2e-4)
    assert np.all(np.abs(U / I) < 1e-3) and np.all(rows[:, 7] == 0.0)
    assert want.min() < -0.99                          # (full polarisation at alpha = 90 deg is in the set)
    return Q / I, want


def _isothermal_thick_flux(atm, temperature, cell_depth, distance):
    """Disk-integrated flux of an isothermal, purely absorbing shell that emits between the
    sphere r_cd = radial[cell_depth] (black, not emitting) and r_top: every ray's emergent
    intensity is B (1 - exp(-kappa s)), s its path through the emitting shell -- the whole
    chord for rays that miss the r_cd sphere (optically thick: B), and sqrt(r_top^2 - b^2) -
    sqrt(r_cd^2 - b^2) for impact parameters b < r_cd.  F = (B / d^2) [pi r_top^2 -
    int_0^r_cd exp(-kappa s(b)) 2 pi b db], by quadrature (spherical, no plane-parallel step)."""
    from scipy.integrate import quad

    rt, rcd = float(atm["radial"][-1]), float(atm["radial"][cell_depth])
    kappa = float(atm["absorption"][0, 0, 0, 0])
    lam = float(atm["wavelength"][0]) * 1e-6
    B = driver.planck(temperature, lam, 2)
    s = lambda b: math.sqrt(rt * rt - b * b) - math.sqrt(rcd * rcd - b * b)   # noqa: E731
    lost, _ = quad(lambda b: math.exp(-kappa * s(b)) * 2.0 * math.pi * b, 0.0, rcd, epsabs=0, epsrel=1e-12, limit=400)
    return B / distance ** 2 * (math.pi * rt * rt - lost), lost / (math.pi * rt * rt)


def check_isothermal_thick_planet(tmp_path, n, transport_factory=None, grid_factory=None):
    """An isothermal (1500 K), purely absorbing, optically thick atmosphere (radial tau_abs 30)
    as the planet source in imaging_mono: photometry.dat's Stokes I equals the disk-integrated
    flux of _isothermal_thick_flux x 1e-6 within 4 packet-level sigma (same packets rerun with
    the packet moments on); Q = U = V = 0 (thermal peels carry I only); luminosity.dat's emitted
    luminosity is the shell's 4 pi kappa B V (to 1e-2), its emergent column 0 (no packet
    scatters, so none leaves the grid after an interaction: flux_exit, ARTES.f90:953)."""
    T = 1500.0
    atm = synthetic.make_thermal(nr=16, ntheta=6, nphi=8, tau_abs=30.0, tau_sca=0.0, temperature=T, wavelength=(2.0,))
    out = _cli(tmp_path, "hot", atm, n, 5, source="planet", mode="imaging_mono", transport_factory=transport_factory)
    cd = int(open(out / "cell_depth.dat").read().split()[-1])
    cfg = driver.default_config()
    cfg.apply("photon:source", "planet")
    F, lost = _isothermal_thick_flux(atm, T, cd, cfg.distance_planet)
    ph = stats.read_photometry(str(out / "photometry.dat"))
    got = ph[1]
    g = grid_factory(atm)
    cd2, total, _ = g.thermal(0, cfg.thermal_weight, False)
    assert cd2 == cd and 0.0 < lost < 5e-3
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    p = driver.run_params(cfg, det, 0, cell_depth=cd, packet_moments=True)
    res = g.run(p, 0, int(n), 5)
    E = driver.package_energy(cfg, 2.0e-6, float(atm["radial"][-1]), int(n), det.det_phi, emissivity_total=total)
    assert got == pytest.approx(res.det[0, 0].sum() * E * 1e-6, rel=1e-12, abs=0)
    sig = stats.total_sigma_raw(res.totals, int(n))[0] * E * 1e-6
    print("thermal flux: got", got, "want", F * 1e-6, "sigma", sig, "lost", lost)
    assert abs(got - F * 1e-6) <= 4.0 * sig, (got, F * 1e-6, sig)
    assert sig < 3e-3 * got * math.sqrt(4e6 / n)
    assert np.all(ph[3:8:2] == 0.0)
    lum = [[float(v) for v in l.split()] for l in open(out / "luminosity.dat").read().splitlines()
           if l.strip() and "#" not in l]
    rt, rcd = float(atm["radial"][-1]), float(atm["radial"][cd])
    kappa = float(atm["absorption"][0, 0, 0, 0])
    emitted = 4.0 * math.pi * kappa * driver.planck(T, 2.0e-6, 2) * (4.0 / 3.0) * math.pi * (rt ** 3 - rcd ** 3) * 1e-6
    assert lum[0][1] == pytest.approx(emitted, rel=1e-2) and lum[0][2] == 0.0
    return got, F * 1e-6, sig


def _gpu_grid(atm):
    from artes_amd.engine import Grid

    return Grid(atm, device=0)


def test_gpu_lambert_sphere_phase_curve(require_gpu, tmp_path):
    check_lambert_phase_curve(tmp_path, 10**6, None, _gpu_grid)


def test_gpu_thin_rayleigh_phase_curve_polarisation(require_gpu, tmp_path):
    check_thin_rayleigh_phase_polarisation(tmp_path, 2 * 10**5, None)


def test_gpu_isothermal_thick_planet_flux(require_gpu, tmp_path):
    check_isothermal_thick_planet(tmp_path, 2 * 10**7, None, _gpu_grid)

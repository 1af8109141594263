"""Mie opacity generator (artes_amd.mie, restating python/opacityMie.py with its missing
ComputePart solver replaced by Lorenz-Mie theory).  Parity unpinned against the
reference (no ComputePart output exists); pinned here by Mie theory's known answers."""

import math
import os

import numpy as np
import pytest

from artes_amd import atmosphere, mie, opacity

RI = "/root/reference/dat/refractive_index"
need_ri = pytest.mark.skipif(not os.path.isdir(RI), reason="reference refractive-index tables not present")


def test_bohren_huffman_worked_example():
    # Bohren & Huffman (1983) App. A sample run: m = 1.55, radius 0.525, wavelength 0.6328
    x = 2 * math.pi * 0.525 / 0.6328
    qext, qsca, _, s1, _ = mie.bhmie([x], 1.55, [-1.0])
    assert qext[0] == pytest.approx(3.1054, abs=1e-4)
    assert qsca[0] == pytest.approx(3.1054, abs=1e-4)
    assert 4 * abs(s1[0, 0]) ** 2 / x ** 2 == pytest.approx(2.9253, abs=1e-4)    # Qback


def test_rayleigh_limit():
    m = 1.5 + 0.1j
    x = np.array([1e-3, 3e-3])
    qext, qsca, g, _, _ = mie.bhmie(x, m, [1.0])
    alpha = (m * m - 1) / (m * m + 2)
    np.testing.assert_allclose(qsca, 8 / 3 * x ** 4 * abs(alpha) ** 2, rtol=1e-4)
    np.testing.assert_allclose(qext - qsca, 4 * x * alpha.imag, rtol=1e-4)
    assert np.all(np.abs(g) < 1e-4)
    # dipole matrix: F12/F11 = -sin^2/(1+cos^2), full polarisation at 90 degrees
    mu = np.cos(np.radians([30.0, 90.0, 150.0]))
    _, _, _, s1, s2 = mie.bhmie([1e-3], 1.33, mu)
    f = mie.amplitude_to_matrix(s1, s2)[0]
    np.testing.assert_allclose(f[1] / f[0], -(1 - mu ** 2) / (1 + mu ** 2), atol=1e-6)
    np.testing.assert_allclose(f[3] / f[0], 2 * mu / (1 + mu ** 2), atol=1e-6)


def test_extinction_paradox():
    qext, qsca, g, _, _ = mie.bhmie([2000.0], 1.33 + 0.05j, [1.0])
    # 2 plus the edge (glory/surface-wave) term 1.9923 x^(-2/3) (Nussenzveig & Wiscombe 1980)
    assert qext[0] == pytest.approx(2.0 + 1.9923 * 2000.0 ** (-2 / 3), abs=1e-3)
    assert qsca[0] < qext[0] and g[0] > 0.9


@pytest.mark.parametrize("x,m", [(0.7, 1.33 + 0.0j), (5.0, 1.5 + 0.01j), (30.0, 1.65 + 0.3j), (80.0, 2.0 + 1.0j)])
def test_sum_rules(x, m):
    """Optical theorem, Csca = k^-2 int S11 dOmega, g from the phase function, and the
    single-sphere identity F11^2 = F12^2 + F33^2 + F34^2."""
    nq = 4000
    mu, wq = np.polynomial.legendre.leggauss(nq)
    qext, qsca, g, s1, s2 = mie.bhmie([x], m, np.concatenate([[1.0], mu]))
    assert qext[0] == pytest.approx(4 / x ** 2 * s1[0, 0].real, rel=1e-10)
    assert s1[0, 0] == pytest.approx(s2[0, 0], rel=1e-12)
    f = mie.amplitude_to_matrix(s1[:, 1:], s2[:, 1:])[0]
    assert 2 / x ** 2 * np.sum(wq * f[0]) == pytest.approx(qsca[0], rel=1e-8)
    assert np.sum(wq * f[0] * mu) / np.sum(wq * f[0]) == pytest.approx(g[0], rel=1e-8)
    np.testing.assert_allclose(f[0] ** 2, f[1] ** 2 + f[3] ** 2 + f[4] ** 2, rtol=1e-9)
    if m.imag == 0:
        assert qext[0] == pytest.approx(qsca[0], rel=1e-12)


def test_size_distributions():
    r, w = mie.size_distribution(4000, r_eff=1.4, v_eff=0.05)
    reff = np.sum(w * r ** 3) / np.sum(w * r ** 2)
    veff = np.sum(w * (r - reff) ** 2 * r ** 2) / (reff ** 2 * np.sum(w * r ** 2))
    assert reff == pytest.approx(1.4, rel=1e-5) and veff == pytest.approx(0.05, rel=1e-4)
    r, w = mie.size_distribution(2000, amin=0.1, amax=5.0, apow=-3.5)
    assert r[0] == pytest.approx(0.1) and r[-1] == pytest.approx(5.0)
    exact = (5.0 ** -2.5 - 0.1 ** -2.5) / -2.5
    assert np.sum(w) == pytest.approx(exact, rel=1e-5)


def test_distribution_opacity_and_matrix():
    table = (np.array([0.5, 2.0]), np.array([1.5, 1.5]), np.array([1e-3, 1e-3]))
    op, sc = mie.mie_opacity(table, [1.0], density=2.0, nr=200, r_eff=0.8, v_eff=0.1)
    op1, _ = mie.mie_opacity(table, [1.0], density=1.0, nr=200, r_eff=0.8, v_eff=0.1)
    assert op.shape == (4, 1) and sc.shape == (180, 16, 1)
    np.testing.assert_allclose(op[1:] * 2.0, op1[1:], rtol=1e-12)    # per gram of particles
    assert op[1, 0] == pytest.approx(op[2, 0] + op[3, 0]) and 0 < op[2, 0] < op[3, 0]
    ang = (np.arange(180) + 0.5) * math.pi / 180
    assert 2 * math.pi * opacity.simps_avg(sc[:, 0, 0] * np.sin(ang), ang) == pytest.approx(1.0, rel=1e-12)
    np.testing.assert_array_equal(sc[:, 1], sc[:, 4])
    np.testing.assert_array_equal(sc[:, 11], -sc[:, 14])
    np.testing.assert_array_equal(sc[:, 0], sc[:, 5])
    # a size distribution depolarises: F11^2 >= F12^2 + F33^2 + F34^2
    assert np.all(sc[:, 0] ** 2 + 1e-30 >= sc[:, 1] ** 2 + sc[:, 10] ** 2 + sc[:, 11] ** 2)
    # narrow distribution -> single sphere
    r0 = 0.8
    opn, _ = mie.mie_opacity(table, [1.0], nr=400, r_eff=r0, v_eff=1e-4)
    qext = mie.bhmie([2 * math.pi * r0], 1.5 + 1e-3j, [1.0])[0][0]
    assert opn[1, 0] == pytest.approx(qext * 3 / (4 * r0 * 1e-4), rel=1e-2)   # 1 % spread in r


MU = np.cos((np.arange(180) + 0.5) * math.pi / 180.0)


@pytest.mark.parametrize("m", [1.5 + 0.01j, 1.33 + 1e-4j, 1.7 + 0.1j])
def test_coated_sphere_limits(m):
    """BHCOAT (Bohren & Huffman 1983, App. B) against its exact limits: equal core and
    mantle indices = a homogeneous sphere of the outer size; a vacuum mantle = a homogeneous
    sphere of the core size (efficiencies scale with the area); a vanishing vacuum core = a
    homogeneous sphere of the outer size."""
    y = np.array([0.3, 2.0, 8.0, 25.0])
    qe, qs, s1, s2 = mie.bhcoat(0.6 * y, y, m, m, MU)
    qe0, qs0, _, t1, t2 = mie.bhmie(y, m, MU)
    np.testing.assert_allclose(qe, qe0, rtol=1e-7)
    np.testing.assert_allclose(qs, qs0, rtol=1e-7)
    np.testing.assert_allclose(s1, t1, rtol=0, atol=1e-7 * np.abs(t1).max())
    np.testing.assert_allclose(s2, t2, rtol=0, atol=1e-7 * np.abs(t2).max())
    x = 0.7 * y
    qe, qs, s1, _ = mie.bhcoat(x, y, m, 1.0, MU)
    qe0, qs0, _, t1, _ = mie.bhmie(x, m, MU)
    np.testing.assert_allclose(qe * y ** 2, qe0 * x ** 2, rtol=1e-9)
    np.testing.assert_allclose(s1, t1, rtol=0, atol=1e-9 * np.abs(t1).max())
    qe, qs, _, _ = mie.bhcoat(1e-4 * y, y, 1.0, m, MU)
    qe0, qs0, _, _, _ = mie.bhmie(y, m, MU)
    np.testing.assert_allclose(qe, qe0, rtol=1e-7)
    np.testing.assert_allclose(qs, qs0, rtol=1e-7)


@pytest.mark.parametrize("y", [0.5, 3.0, 15.0])
def test_coated_sphere_energy_and_optical_theorem(y):
    qe, qs, s1, _ = mie.bhcoat([0.5 * y], [y], 1.0, 1.5, [1.0])      # non-absorbing mantle
    assert qe[0] == pytest.approx(qs[0], rel=1e-12)
    assert qe[0] == pytest.approx(4.0 / y ** 2 * s1[0, 0].real, rel=1e-12)   # optical theorem
    qe, qs, s1, _ = mie.bhcoat([0.5 * y], [y], 1.0, 1.5 + 0.05j, [1.0])
    assert qe[0] > qs[0] > 0.0                                          # absorption
    assert qe[0] == pytest.approx(4.0 / y ** 2 * s1[0, 0].real, rel=1e-10)


@pytest.mark.parametrize("m", [2.0 + 1.0j, 3.0 + 3.0j, 1.8 + 0.5j])
def test_coated_sphere_absorbing_mantle(m):
    """Strongly absorbing mantles at size parameters up to 100 (BHCOAT's upward chi
    recurrences overflow there and returned NaN): the equal-index and vanishing-core limits
    are the homogeneous outer sphere, a vacuum mantle the homogeneous core, and a deep void
    inside an opaque mantle is invisible; everything finite, extinction >= scattering, and
    the optical theorem holds."""
    y = np.array([1.0, 10.0, 25.0, 60.0, 100.0])
    qe, qs, s1, s2 = mie.bhcoat(0.6 * y, y, m, m, MU)
    qe0, qs0, _, t1, t2 = mie.bhmie(y, m, MU)
    np.testing.assert_allclose(qe, qe0, rtol=1e-9)
    np.testing.assert_allclose(qs, qs0, rtol=1e-9)
    np.testing.assert_allclose(s1, t1, rtol=0, atol=1e-9 * np.abs(t1).max())
    np.testing.assert_allclose(s2, t2, rtol=0, atol=1e-9 * np.abs(t2).max())
    qe, qs, s1, _ = mie.bhcoat(1e-4 * y, y, 1.0, m, MU)                      # vanishing vacuum core
    np.testing.assert_allclose(qe, qe0, rtol=1e-7)
    np.testing.assert_allclose(qs, qs0, rtol=1e-7)
    qe, qs, s1, _ = mie.bhcoat(0.7 * y, y, m, 1.0, MU)                       # vacuum mantle
    qc, qsc, _, tc, _ = mie.bhmie(0.7 * y, m, MU)
    np.testing.assert_allclose(qe * y ** 2, qc * (0.7 * y) ** 2, rtol=1e-9)
    np.testing.assert_allclose(s1, tc, rtol=0, atol=1e-9 * np.abs(tc).max())
    qe, qs, s1, s2 = mie.bhcoat(0.5 * y, y, 1.0, m, MU)                      # a void in the absorber
    assert np.all(np.isfinite(s1)) and np.all(np.isfinite(s2))
    assert np.all(qe >= qs) and np.all(qs > 0)
    _, _, f1, _ = mie.bhcoat(0.5 * y, y, 1.0, m, [1.0])
    np.testing.assert_allclose(qe, 4.0 / y ** 2 * f1[:, 0].real, rtol=1e-10)   # optical theorem
    big = 2.0 * m.imag * 0.5 * y > 60.0                                      # exp(-2 Im(m) (y - x)) < 1e-26
    np.testing.assert_allclose(qe[big], qe0[big], rtol=1e-10)


def test_hollow_spheres_absorbing_index():
    """The distribution of hollow spheres of a strongly absorbing material (fmax = 0.8): finite
    opacities and matrices (these were NaN)."""
    for n_k in (3.0 + 3.0j, 1.8 + 0.5j):
        ri = (np.array([0.3, 1.0]), np.array([n_k.real] * 2), np.array([n_k.imag] * 2))
        op, sc = mie.mie_opacity(ri, [0.5], nr=40, fmax=0.8, nf=6)
        assert np.all(np.isfinite(op)) and np.all(np.isfinite(sc)) and op[2, 0] > 0 and op[3, 0] > 0


def test_hollow_sphere_distribution():
    """DHS (fmax > 0, opacityMie.py:15,20): the fmax -> 0 limit is the homogeneous
    distribution; voids change the matrix smoothly; material mass (and so the opacity per
    gram's normalisation) is that of the solid particles."""
    ri = (np.array([0.5, 2.0]), np.array([1.5, 1.5]), np.array([1e-3, 1e-3]))
    kw = dict(density=1.0, nr=40, r_eff=0.5, v_eff=0.1)
    op0, sc0 = mie.mie_opacity(ri, [0.8], **kw)
    # the void shifts the particle's outer radius by ~f/3 (material volume kept): the
    # departure from the homogeneous distribution is first order in fmax and vanishes with it
    d = []
    for fmax in (1e-5, 1e-6):
        op1, sc1 = mie.mie_opacity(ri, [0.8], fmax=fmax, nf=4, **kw)
        np.testing.assert_allclose(op1, op0, rtol=20 * fmax)
        d.append(np.abs(sc1 - sc0).max() / np.abs(sc0).max())
    assert d[0] < 1e-4 and 7.0 < d[0] / d[1] < 13.0, d
    op8, sc8 = mie.mie_opacity(ri, [0.8], fmax=0.8, nf=10, **kw)
    assert op8[1, 0] > 0 and op8[3, 0] > 0 and op8[1, 0] != pytest.approx(op0[1, 0], rel=1e-3)
    # normalised matrix: 2 pi int P11 sin = 1 (atmosphere.py:60-65 conventions)
    ang = (np.arange(180) + 0.5) * math.pi / 180
    assert 2 * math.pi * np.sum(sc8[:, 0, 0] * np.sin(ang)) * math.pi / 180 == pytest.approx(1.0, rel=2e-3)
    np.testing.assert_allclose(mie.dhs_fractions(4, 0.8), [0.1, 0.3, 0.5, 0.7])
    with pytest.raises(ValueError):
        mie.dhs_fractions(0, 0.5)


@need_ri
def test_script_defaults_into_atmosphere(tmp_path):
    """opacityMie.py's defaults (ammonia ice, r_eff 1.4, v_eff 0.05, 1.6 micron) into
    atmosphere.py's cloud branch."""
    d = tmp_path / "clouds"
    (d / "opacity").mkdir(parents=True)
    mie.write_mie_opacity(str(d / "opacity" / "ammonia.fits"), os.path.join(RI, "ammonia_ice.dat"), nr=300)
    op, sc = opacity.read_opacity_fits(str(d / "opacity" / "ammonia.fits"))
    assert op[0, 0] == pytest.approx(1.6) and op[2, 0] > 0 and op[3, 0] > 100 * op[2, 0]
    assert sc[0, 0, 0] > 100 * sc[90, 0, 0]           # forward diffraction peak
    (d / "atmosphere.in").write_text(
        "[grid]\nradius: 1.\nradial: 10., 20.\ntheta:\nphi:\n\n[composition]\ngas: off\n"
        "ring:\nfits01: ammonia.fits\nopacity01: 1, 1e-6, 1, nr, 0, ntheta, 0, nphi\n")
    atm = atmosphere.build(str(d))
    ks = atm["scattering"]
    assert ks.shape[-1] == 2 and np.all(ks[..., 0] == 0) and np.all(ks[..., 1] > 0)
    # kg m-3 times m2 kg-1: the cloud layer's extinction is density x mass opacity
    np.testing.assert_allclose(ks[..., 1], 1e-3 * op[3, 0] / 10.0, rtol=1e-12)

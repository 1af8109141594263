"""Mie opacity generator: restatement of ``python/opacityMie.py`` without its external
solver.

The reference script writes ``mie.in`` / ``wavelength.dat`` and runs the prebuilt
``bin/ComputePartLinux`` (``opacityMie.py:48-105``), which is not part of the reference
checkout (and prebuilt reference binaries are never run here anyway).  This module
replaces that solver with its published algorithm -- Lorenz-Mie theory for homogeneous
spheres in the Bohren & Huffman (1983, App. A) formulation -- averaged over the same two
size distributions the script configures:

* ``r_eff > 0``: the two-parameter gamma distribution of Hansen & Travis (1974, eq. 2.56),
  ``n(r) ~ r**((1 - 3 v_eff) / v_eff) * exp(-r / (r_eff v_eff))``
  (``opacityMie.py:21-22``, "overrules amin, amax, apow");
* otherwise the power law ``n(a) ~ a**apow`` on ``[amin, amax]`` (``opacityMie.py:17-19``);

with ``nr`` radii (``opacityMie.py:14``) log-spaced over the distribution and
trapezoidal weights in ``ln r``.  Then exactly the script's own post-processing: the
6 -> 16 element expansion (``opacityMie.py:116-131``) and the per-wavelength
``2 pi simps(P11 sin)`` normalisation on the bin-centre angles
(``opacityMie.py:133-144``), whose ``(i + 0.5)`` degrees also fix where the 180 rows
are evaluated here.

Conventions: the six elements are F11, F12, F22, F33, F34, F44 in Bohren & Huffman's
sign convention -- the one the reference's Rayleigh generator uses (F12 < 0 at 90
degrees, ``opacityRayleigh.py:97-108``).  Refractive indices are read from the
reference's ``dat/refractive_index/*.dat`` format (wavelength [micron], n, k) and
interpolated linearly in log wavelength (n) and log-log (k), held constant outside the
tabulated range.

**Parity unpinned**: ComputePart's output is not available, so no reference number
exists for this generator.  The solver is pinned instead by Mie theory's own
known answers (tests/test_mie.py): the Rayleigh limit, the extinction paradox, the
optical theorem, the ``Csca = (1/k^2) int S11 dOmega`` identity, single-sphere
polarisation identities and the Bohren & Huffman worked example.

The distribution of hollow spheres (DHS; ``fmax > 0`` with ``nf`` volume fractions,
``opacityMie.py:15,20``) follows its published definition (Min, Hovenier & de Koter
2005, A&A 432, 909): every particle of the size distribution becomes a sphere with a
central vacuum inclusion whose volume fraction f is uniform on ``[0, fmax]``, the material
volume kept equal to the solid sphere's (outer radius ``r / (1 - f)**(1/3)``, core
``f**(1/3)`` of that), and the cross sections and matrices are averaged over f with the
midpoint rule on ``nf`` points.  The coated spheres are solved with Bohren & Huffman's
coated-sphere coefficients in Yang's (2003) bounded recurrences (absorbing mantles included).  ComputePart's own f quadrature is not known (its
binary is absent), so this path is parity-unpinned too; tests/test_mie.py pins the
coated-sphere solver by its limits (equal indices, vanishing core, vacuum mantle), the
optical theorem and energy conservation, and DHS by its ``fmax -> 0`` limit.
"""

from __future__ import annotations

import math

import numpy as np

from .opacity import expand_six_elements, normalize_matrix, wavelength_grid, write_opacity_fits


def read_refractive_index(path: str):
    """``np.loadtxt(riDir+riFile, unpack=True)`` (``opacityMie.py:62``)."""
    wav, n, k = np.loadtxt(path, unpack=True, ndmin=2)
    order = np.argsort(wav)
    return wav[order], n[order], k[order]


def refractive_index_at(table, wavelength) -> np.ndarray:
    """Complex m = n + i k at ``wavelength`` [micron] (see module docstring)."""
    wav, n, k = table
    lw = np.log(np.atleast_1d(np.asarray(wavelength, dtype=np.float64)))
    lt = np.log(wav)
    re = np.interp(lw, lt, n)
    if np.all(k > 0):
        im = np.exp(np.interp(lw, lt, np.log(k)))
    else:
        im = np.interp(lw, lt, k)
    return re + 1j * im


def bhmie(x, m: complex, mu):
    """Lorenz-Mie solution for spheres of size parameters ``x`` (array) and relative
    refractive index ``m`` at scattering-angle cosines ``mu``.

    Returns ``qext, qsca, g, s1, s2`` with ``s1``/``s2`` of shape ``(len(x), len(mu))``.
    Logarithmic derivative D_n(mx) by downward recurrence, Riccati-Bessel functions and
    the angular functions pi_n, tau_n by upward recurrence, series truncated at
    Wiscombe's ``x + 4 x^(1/3) + 2`` (Bohren & Huffman 1983, App. A).  All sizes are
    advanced together; a size stops accumulating (and its recurrences freeze) once its
    own truncation order is passed.
    """
    x = np.atleast_1d(np.asarray(x, dtype=np.float64))
    mu = np.atleast_1d(np.asarray(mu, dtype=np.float64))
    if np.any(x <= 0):
        raise ValueError("size parameters must be positive")
    m = complex(m)
    y = m * x
    nstop = np.floor(x + 4.0 * np.cbrt(x) + 2.0).astype(np.int64)
    nmax = int(nstop.max())
    nmx = int(max(nmax, np.abs(y).max())) + 15

    # D_n(y), n = 0..nmax, downward from nmx (stable for every size at once)
    d = np.zeros((nmax + 1, x.size), dtype=np.complex128)
    dn = np.zeros(x.size, dtype=np.complex128)
    for n in range(nmx, 0, -1):
        dn = n / y - 1.0 / (dn + n / y)
        if n - 1 <= nmax:
            d[n - 1] = dn

    psi0, psi1 = np.cos(x), np.sin(x)
    chi0, chi1 = -np.sin(x), np.cos(x)
    xi1 = psi1 - 1j * chi1
    pi0 = np.zeros(mu.size)
    pi1 = np.ones(mu.size)
    s1 = np.zeros((x.size, mu.size), dtype=np.complex128)
    s2 = np.zeros((x.size, mu.size), dtype=np.complex128)
    qext = np.zeros(x.size)
    qsca = np.zeros(x.size)
    gsum = np.zeros(x.size)
    an1 = np.zeros(x.size, dtype=np.complex128)
    bn1 = np.zeros(x.size, dtype=np.complex128)
    for n in range(1, nmax + 1):
        act = n <= nstop
        en = float(n)
        fn = (2.0 * en + 1.0) / (en * (en + 1.0))
        psi = (2.0 * en - 1.0) * psi1 / x - psi0
        chi = (2.0 * en - 1.0) * chi1 / x - chi0
        xi = psi - 1j * chi
        da = d[n] / m + en / x
        db = d[n] * m + en / x
        an = np.where(act, (da * psi - psi1) / (da * xi - xi1), 0.0)
        bn = np.where(act, (db * psi - psi1) / (db * xi - xi1), 0.0)
        qext += (2.0 * en + 1.0) * (an.real + bn.real)
        qsca += (2.0 * en + 1.0) * (np.abs(an) ** 2 + np.abs(bn) ** 2)
        if n > 1:
            gsum += ((en - 1.0) * (en + 1.0) / en) * (an1 * an.conj() + bn1 * bn.conj()).real
        gsum += ((2.0 * en + 1.0) / (en * (en + 1.0))) * (an * bn.conj()).real
        # angular functions at this order
        tau = en * mu * pi1 - (en + 1.0) * pi0
        s1 += fn * (an[:, None] * pi1[None, :] + bn[:, None] * tau[None, :])
        s2 += fn * (an[:, None] * tau[None, :] + bn[:, None] * pi1[None, :])
        pi_next = ((2.0 * en + 1.0) * mu * pi1 - (en + 1.0) * pi0) / en
        pi0, pi1 = pi1, pi_next
        psi0 = np.where(act, psi1, psi0)
        psi1 = np.where(act, psi, psi1)
        chi0 = np.where(act, chi1, chi0)
        chi1 = np.where(act, chi, chi1)
        xi1 = psi1 - 1j * chi1
        an1, bn1 = an, bn
    qsca *= 2.0 / (x * x)
    qext *= 2.0 / (x * x)
    g = 4.0 * gsum / (x * x * qsca)
    return qext, qsca, g, s1, s2


def _logderiv_down(z, nmax: int):
    """D_n(z) = psi_n'(z) / psi_n(z), n = 0..nmax, for complex z (one per size), by downward
    recurrence from max(nmax, |z|) + 15 (stable for any z, as in :func:`bhmie`)."""
    nmx = int(max(nmax, np.abs(z).max())) + 15
    d = np.zeros((nmax + 1, z.size), dtype=np.complex128)
    dn = np.zeros(z.size, dtype=np.complex128)
    for n in range(nmx, 0, -1):
        dn = n / z - 1.0 / (dn + n / z)
        if n - 1 <= nmax:
            d[n - 1] = dn
    return d


def bhcoat(x, y, m1: complex, m2: complex, mu):
    """Coated spheres: core size parameters ``x`` and index ``m1``, outer size parameters
    ``y`` (arrays of equal length) and mantle index ``m2``, at scattering-angle cosines
    ``mu``.  Returns ``qext, qsca, s1, s2`` as :func:`bhmie` (without g).

    The coefficients of Bohren & Huffman's coated sphere (1983, sec. 8.1), evaluated with
    bounded quantities only (Yang 2003, Appl. Opt. 42, 1710): in the mantle the radial
    function is psi_n(z) + c xi_n(z), z = m2 k r; matching the core's log-derivative D_n(m1 x)
    at the interface fixes c, and the mantle's log-derivative at its outer surface is
    H_n = (D_n(z2) + w D3_n(z2)) / (1 + w),  w = -(D_n(z1) - H_t) / (D3_n(z1) - H_t) Q_n,
    with H_t = (m2/m1) D_n(m1 x) (a_n) or (m1/m2) D_n(m1 x) (b_n), z1 = m2 x, z2 = m2 y,
    D3 = xi'/xi and Q_n = (psi_n/xi_n)(z1) / (psi_n/xi_n)(z2).  D_n by downward recurrence,
    psi_n xi_n and D3_n = D_n + i/(psi_n xi_n) upward from closed forms at n = 0, and Q_n as
    a running product -- none of them grows with the mantle's absorption, so an absorbing
    mantle around a deep core gives the homogeneous outer sphere (|Q_n| ~ exp(-2 Im(m2)(y - x)))
    instead of the overflow of BHCOAT's upward chi recurrences.  The series is truncated at
    ``y + 4 y^(1/3) + 2``.
    """
    x = np.atleast_1d(np.asarray(x, dtype=np.float64))
    y = np.atleast_1d(np.asarray(y, dtype=np.float64))
    mu = np.atleast_1d(np.asarray(mu, dtype=np.float64))
    if np.any(x <= 0) or np.any(y < x):
        raise ValueError("need 0 < x <= y")
    m1, m2 = complex(m1), complex(m2)
    if m1.imag < 0 or m2.imag < 0:
        raise ValueError("refractive indices n + ik need k >= 0")
    nstop = np.floor(y + 4.0 * np.cbrt(y) + 2.0).astype(np.int64)
    nmax = int(nstop.max())
    zc, z1, z2 = m1 * x + 0j, m2 * x + 0j, m2 * y + 0j
    dc, d1, d2 = _logderiv_down(zc, nmax), _logderiv_down(z1, nmax), _logderiv_down(z2, nmax)
    # n = 0: psi_0 xi_0 = (1 - e^{2iz}) / 2, D3_0 = i, Q_0 = (e^{2i z1} - 1) / (e^{2i z2} - 1) e^{2i (z2 - z1)}
    e1, e2 = np.exp(2j * z1), np.exp(2j * z2)
    px1, px2 = 0.5 * (1.0 - e1), 0.5 * (1.0 - e2)
    d31 = np.full(x.size, 1j)
    d32 = np.full(x.size, 1j)
    q = (e1 - 1.0) / (e2 - 1.0) * np.exp(2j * (z2 - z1))
    psi0y, psi1y = np.cos(y), np.sin(y)
    chi0y, chi1y = -np.sin(y), np.cos(y)
    xi1y = psi1y - 1j * chi1y
    qext = np.zeros(x.size)
    qsca = np.zeros(x.size)
    pi0 = np.zeros(mu.size)
    pi1 = np.ones(mu.size)
    s1 = np.zeros((x.size, mu.size), dtype=np.complex128)
    s2 = np.zeros((x.size, mu.size), dtype=np.complex128)
    for n in range(1, nmax + 1):
        act = n <= nstop
        rn = float(n)
        # step psi xi, D3 and Q from n-1 to n (factors with D_{n-1}, D3_{n-1})
        f1a, f1b = rn / z1 - d1[n - 1], rn / z1 - d31
        f2a, f2b = rn / z2 - d2[n - 1], rn / z2 - d32
        px1, px2 = px1 * f1a * f1b, px2 * f2a * f2b
        q = q * (f1a / f1b) * (f2b / f2a)
        d31 = d1[n] + 1j / px1
        d32 = d2[n] + 1j / px2
        ht_a, ht_b = (m2 / m1) * dc[n], (m1 / m2) * dc[n]
        wa = -(d1[n] - ht_a) / (d31 - ht_a) * q
        wb = -(d1[n] - ht_b) / (d31 - ht_b) * q
        ha = (d2[n] + wa * d32) / (1.0 + wa)
        hb = (d2[n] + wb * d32) / (1.0 + wb)
        psiy = (2.0 * rn - 1.0) * psi1y / y - psi0y
        chiy = (2.0 * rn - 1.0) * chi1y / y - chi0y
        xiy = psiy - 1j * chiy
        ca = ha / m2 + rn / y
        cb = m2 * hb + rn / y
        an = np.where(act, (ca * psiy - psi1y) / (ca * xiy - xi1y), 0.0)
        bn = np.where(act, (cb * psiy - psi1y) / (cb * xiy - xi1y), 0.0)
        qsca += (2.0 * rn + 1.0) * (np.abs(an) ** 2 + np.abs(bn) ** 2)
        qext += (2.0 * rn + 1.0) * (an.real + bn.real)
        fn = (2.0 * rn + 1.0) / (rn * (rn + 1.0))
        tau = rn * mu * pi1 - (rn + 1.0) * pi0
        s1 += fn * (an[:, None] * pi1[None, :] + bn[:, None] * tau[None, :])
        s2 += fn * (an[:, None] * tau[None, :] + bn[:, None] * pi1[None, :])
        pi_next = ((2.0 * rn + 1.0) * mu * pi1 - (rn + 1.0) * pi0) / rn
        pi0, pi1 = pi1, pi_next
        psi0y = np.where(act, psi1y, psi0y)
        psi1y = np.where(act, psiy, psi1y)
        chi0y = np.where(act, chi1y, chi0y)
        chi1y = np.where(act, chiy, chi1y)
        xi1y = psi1y - 1j * chi1y
    qsca *= 2.0 / (y * y)
    qext *= 2.0 / (y * y)
    if not (np.all(np.isfinite(qext)) and np.all(np.isfinite(qsca)) and np.all(np.isfinite(s1))
            and np.all(np.isfinite(s2))):
        raise FloatingPointError("bhcoat: non-finite result")
    return qext, qsca, s1, s2


def dhs_fractions(nf: int, fmax: float) -> np.ndarray:
    """Vacuum volume fractions of the DHS average: midpoints of ``nf`` equal bins of [0, fmax]."""
    if nf < 1 or not 0.0 <= fmax < 1.0:
        raise ValueError("need nf >= 1 and 0 <= fmax < 1")
    return fmax * (np.arange(nf) + 0.5) / nf


def amplitude_to_matrix(s1, s2):
    """Six independent elements (F11, F12, F22, F33, F34, F44) of a sphere's
    scattering matrix from its amplitudes (Bohren & Huffman eq. 4.77)."""
    a1, a2 = np.abs(s1) ** 2, np.abs(s2) ** 2
    s21 = s2 * s1.conj()
    f11 = 0.5 * (a2 + a1)
    f12 = 0.5 * (a2 - a1)
    f33 = s21.real
    f34 = s21.imag
    return np.stack([f11, f12, f11, f33, f34, f33], axis=-2)


def size_distribution(nr: int, amin: float = 0.1, amax: float = 5.0, apow: float = 0.0,
                      r_eff: float = 0.0, v_eff: float = 0.0):
    """Radii [micron] and number weights n(r) dr of the configured distribution
    (``opacityMie.py:14-22``): trapezoidal in ln r over ``nr`` log-spaced radii."""
    if nr < 2:
        raise ValueError("nr must be at least 2")
    if r_eff > 0.0:
        if not 0.0 < v_eff < 0.5:
            raise ValueError("v_eff must be in (0, 0.5) for the gamma distribution")
        from scipy.stats import gamma
        shape = (1.0 - 3.0 * v_eff) / v_eff + 1.0      # gamma pdf shape in r
        scale = r_eff * v_eff
        lo, hi = gamma.ppf([1e-10, 1.0 - 1e-12], shape, scale=scale)
        r = np.exp(np.linspace(math.log(lo), math.log(hi), nr))
        ln_n = (shape - 1.0) * np.log(r) - r / scale
        nd = np.exp(ln_n - ln_n.max())
    else:
        if not 0.0 < amin < amax:
            raise ValueError("need 0 < amin < amax")
        r = np.exp(np.linspace(math.log(amin), math.log(amax), nr))
        nd = r ** apow
    w = np.full(nr, math.log(r[1] / r[0]))
    w[0] *= 0.5
    w[-1] *= 0.5
    return r, nd * r * w                                   # n(r) dr = n(r) r dln r


def _particle(r, k: float, m: complex, mu, fracs):
    """Size-resolved (qext, qsca, F[180 or len(mu)][6] per size) of solid spheres of radius
    ``r`` [micron] (fracs None) or of their DHS average: cross-section efficiencies refer to
    the solid sphere's area pi r^2, so the caller's size weights stay those of the solid
    particles (the DHS keeps the material volume)."""
    if fracs is None:
        qext, qsca, _, s1, s2 = bhmie(k * r, m, mu)
        return qext, qsca, amplitude_to_matrix(s1, s2)
    qext = np.zeros(r.size)
    qsca = np.zeros(r.size)
    f6 = 0.0
    for f in fracs:
        rout = r / (1.0 - f) ** (1.0 / 3.0)
        if f == 0.0:
            qe, qs, _, s1, s2 = bhmie(k * rout, m, mu)
        else:
            qe, qs, s1, s2 = bhcoat(k * rout * f ** (1.0 / 3.0), k * rout, 1.0 + 0.0j, m, mu)
        area = (rout / r) ** 2                     # pi rout^2 / pi r^2
        qext += qe * area / len(fracs)
        qsca += qs * area / len(fracs)
        f6 = f6 + amplitude_to_matrix(s1, s2) / len(fracs)
    return qext, qsca, f6


def mie_opacity(refractive_index, wavelengths, density: float = 1.0, nr: int = 1000,
                amin: float = 0.1, amax: float = 5.0, apow: float = 0.0, fmax: float = 0.0,
                r_eff: float = 1.4, v_eff: float = 0.05, normalizer: str = "simps", nf: int = 20):
    """``opacityMie.py`` end to end: ``(opacity (4, nwav), scatter (180, 16, nwav))``.

    ``refractive_index`` is a path in the reference's ``.dat`` format or a
    ``(wavelength, n, k)`` tuple.  Opacities are per gram of particles
    [cm2 g-1]: size-averaged cross sections over the size-averaged particle mass
    ``4/3 pi r^3 density``.  ``fmax > 0``: the distribution of hollow spheres with ``nf``
    volume fractions (module docstring).
    """
    fracs = dhs_fractions(nf, fmax) if fmax > 0.0 else None
    table = read_refractive_index(refractive_index) if isinstance(refractive_index, str) \
        else tuple(np.asarray(a, dtype=np.float64) for a in refractive_index)
    wavelengths = np.atleast_1d(np.asarray(wavelengths, dtype=np.float64))
    r, wn = size_distribution(nr, amin, amax, apow, r_eff, v_eff)
    mass = np.sum(wn * (4.0 / 3.0) * math.pi * (r * 1e-4) ** 3 * density)       # g
    theta = (np.arange(180) + 0.5) * math.pi / 180.0
    mu = np.cos(theta)
    nwav = wavelengths.size
    opacity = np.zeros((4, nwav))
    six = np.zeros((180, 6, nwav))
    for j, (w, m) in enumerate(zip(wavelengths, refractive_index_at(table, wavelengths))):
        k = 2.0 * math.pi / w
        qext, qsca, f6 = _particle(r, k, m, mu, fracs)
        area = math.pi * (r * 1e-4) ** 2                                        # cm2
        c_ext = np.sum(wn * qext * area)
        c_sca = np.sum(wn * qsca * area)
        opacity[0, j] = w
        opacity[1, j] = c_ext / mass
        opacity[3, j] = c_sca / mass
        opacity[2, j] = opacity[1, j] - opacity[3, j]
        f = np.einsum("s,sea->ae", wn, f6)
        # per steradian, normalised to the size-averaged scattering cross section
        six[:, :, j] = f / (k * k * np.sum(wn * qsca * math.pi * r * r))
    return opacity, normalize_matrix(expand_six_elements(six), normalizer)


def write_mie_opacity(path: str, riFile: str, wavelength_min: float = 1.6, wavelength_max: float = 1.6,
                      step: float = 1.0, **kw) -> str:
    """The script's defaults: manual wavelength range (``opacityMie.py:31-35``, ``85-88``),
    written as the opacity FITS file ``atmosphere.py`` reads (``opacityMie.py:146-157``)."""
    opacity, scatter = mie_opacity(riFile, wavelength_grid(wavelength_min, wavelength_max, step), **kw)
    write_opacity_fits(path, opacity, scatter)
    return path

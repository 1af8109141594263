"""Opacity / scattering-matrix generators (Python 3 restatement of the reference's
``python/opacityIsotropic.py``, ``opacityHenyeyGreenstein.py`` and ``opacityRayleigh.py``).

Every generator returns ``(opacity, scatter)``:

* ``opacity``  shape ``(4, nwav)``: wavelength [micron], extinction, absorption,
  scattering [cm2 g-1]  (``opacityRayleigh.py:124-128``)
* ``scatter``  shape ``(180, 16, nwav)``: the 16-element matrix averaged over the
  two edges of each 1-degree bin, ``(M(cos j deg) + M(cos (j+1) deg)) / 2``
  (``opacityRayleigh.py:113-122``, ``opacityHenyeyGreenstein.py:101-109``),
  divided by the generator's own analytic normalisation.

``write_opacity_fits`` stores them as HDU0 / HDU1 exactly like the astropy
``HDUList`` the reference writes.  ``simps_avg`` restates the pre-1.11
``scipy.integrate.simps(y, x)`` (default ``even='avg'``) that ``atmosphere.py:4``
imports; the installed SciPy no longer ships it and its ``simpson`` differs by
~6e-9 relative on these 180-point grids.
"""

from __future__ import annotations

import math

import numpy as np
from scipy.integrate import quad

from . import fitsio


def wavelength_grid(wmin: float, wmax: float, step: float) -> list[float]:
    """``for i in range(int((wavelengthMax-wavelengthMin)/step)+1)`` (``opacityRayleigh.py:40-43``)."""
    return [wmin + float(i) * step for i in range(int((wmax - wmin) / step) + 1)]


def _basic_simps(y, start, stop, x):
    h = np.diff(x)
    sl0 = slice(start, stop, 2)
    sl1 = slice(start + 1, stop + 1, 2)
    sl2 = slice(start + 2, stop + 2, 2)
    h0 = h[sl0]
    h1 = h[sl1]
    hsum = h0 + h1
    hprod = h0 * h1
    h0divh1 = h0 / h1
    tmp = hsum / 6.0 * (y[sl0] * (2 - 1.0 / h0divh1) + y[sl1] * hsum * hsum / hprod + y[sl2] * (2 - h0divh1))
    return np.sum(tmp)


def simps_avg(y, x) -> float:
    """Composite Simpson's rule with SciPy's historical ``even='avg'`` treatment."""
    y = np.asarray(y, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    n = y.shape[0]
    if n % 2 == 1:
        return float(_basic_simps(y, 0, n - 2, x))
    val = 0.0
    last_dx = x[-1] - x[-2]
    val += 0.5 * last_dx * (y[-1] + y[-2])
    result = _basic_simps(y, 0, n - 3, x)
    first_dx = x[1] - x[0]
    val += 0.5 * first_dx * (y[1] + y[0])
    result += _basic_simps(y, 1, n - 2, x)
    val /= 2.0
    result /= 2.0
    return float(result + val)


def _opacity_table(wavelength, absorption, scattering):
    opacity = np.zeros((4, len(wavelength)))
    for i, w in enumerate(wavelength):
        opacity[0, i] = w
        opacity[1, i] = absorption + scattering
        opacity[2, i] = absorption
        opacity[3, i] = scattering
    return opacity


def isotropic(wavelength, absorption: float = 0.0, scattering: float = 1.0):
    """``opacityIsotropic.py:43-60``: P11 = 1/(4 pi), all other elements zero."""
    opacity = _opacity_table(wavelength, absorption, scattering)
    scatter = np.zeros((180, 16, len(wavelength)))
    scatter[:, 0, :] = 1.0 / (4.0 * math.pi)
    return opacity, scatter


def henyey_greenstein(wavelength, g1=0.9, w1=1.0, g2=0.0, w2=0.0, g3=0.0, w3=0.0,
                      p_linear=0.5, p_circular=0.0, skew=0.0,
                      absorption: float = 0.0, scattering: float = 1.0):
    """``opacityHenyeyGreenstein.py:54-119`` (up to three HG lobes, linear/circular polarisation)."""
    opacity = _opacity_table(wavelength, absorption, scattering)

    def hg_p11(theta):
        a = math.cos(theta)
        h = w1 * (1.0 - g1 * g1) / ((1.0 + g1 * g1 - 2.0 * g1 * a) ** 1.5)
        h += w2 * (1.0 - g2 * g2) / ((1.0 + g2 * g2 - 2.0 * g2 * a) ** 1.5)
        h += w3 * (1.0 - g3 * g3) / ((1.0 + g3 * g3 - 2.0 * g3 * a) ** 1.5)
        return h * math.sin(theta)

    def hg_matrix(alpha):
        m = np.zeros(16)
        # the reference feeds cos(angle) into the skew term as if it were an angle
        # (``opacityHenyeyGreenstein.py:83``); kept verbatim
        alpha_f = alpha * (1.0 + 3.13 * skew * math.exp(-7.0 * alpha / math.pi))
        ca = math.cos(alpha_f)
        m[0] = w1 * (1.0 - g1 * g1) / ((1.0 + g1 * g1 - 2.0 * g1 * alpha) ** 1.5)
        m[0] += w2 * (1.0 - g2 * g2) / ((1.0 + g2 * g2 - 2.0 * g2 * alpha) ** 1.5)
        m[0] += w3 * (1.0 - g3 * g3) / ((1.0 + g3 * g3 - 2.0 * g3 * alpha) ** 1.5)
        m[1] = -p_linear * m[0] * (1.0 - alpha * alpha) / (1.0 + alpha * alpha)
        m[4] = m[1]
        m[5] = m[0]
        m[10] = m[0] * (2.0 * alpha) / (1.0 + alpha * alpha)
        m[11] = p_circular * m[5] * (1.0 - ca * ca) / (1.0 + ca * ca)
        m[14] = -m[11]
        m[15] = m[10]
        return m

    norm, _ = quad(hg_p11, 0.0, math.pi)
    norm *= 2.0 * math.pi
    scatter = np.zeros((180, 16, len(wavelength)))
    for j in range(180):
        lo = hg_matrix(math.cos(float(j) * math.pi / 180.0))
        up = hg_matrix(math.cos(float(j + 1) * math.pi / 180.0))
        scatter[j, :, :] = (((lo + up) / 2.0) / norm)[:, None]
    return opacity, scatter


def rayleigh(wavelength, mmw_scat: float = 2.02, depolarization: float = 0.0,
             single_scattering_albedo: float = 1.0):
    """``opacityRayleigh.py:45-122``: H2-like Rayleigh cross-section and depolarised matrix."""
    avogadro = 6.02214129e23
    loschmidt = 2.6867805e19
    gas_mass = mmw_scat / avogadro
    opacity = np.zeros((4, len(wavelength)))
    for i, w in enumerate(wavelength):
        a = 13.58e-5
        b = 7.52e-3
        ri = 1.0 + a + a * b / (w * w)
        rindex = (ri * ri - 1.0) * (ri * ri - 1.0) / ((ri * ri + 2.0) * (ri * ri + 2.0))
        dep = (6.0 + 3.0 * depolarization) / (6.0 - 7.0 * depolarization)
        cross = 24.0 * math.pi ** 3 * rindex * dep / (((w * 1.0e-4) ** 4) * (loschmidt ** 2))
        k_sca = cross / gas_mass
        opacity[0, i] = w
        opacity[1, i] = k_sca / single_scattering_albedo
        opacity[2, i] = k_sca / single_scattering_albedo - k_sca
        opacity[3, i] = k_sca

    delta = (1.0 - depolarization) / (1.0 + depolarization / 2.0)
    delta_p = (1.0 - 2.0 * depolarization) / (1.0 - depolarization)

    def p11(theta):
        a = math.cos(theta)
        return (((a * a + 1.0) * delta) + (1.0 - delta)) * math.sin(theta)

    def matrix(a):
        m = np.zeros(16)
        m[0] = a * a + 1.0
        m[1] = a * a - 1.0
        m[4] = m[1]
        m[5] = m[0]
        m[10] = 2.0 * a
        m[15] = delta_p * m[10]
        m = delta * m
        m[0] = m[0] + (1.0 - delta)
        return m

    norm, _ = quad(p11, 0.0, math.pi)
    norm *= 2.0 * math.pi
    scatter = np.zeros((180, 16, len(wavelength)))
    for j in range(180):
        lo = matrix(math.cos(float(j) * math.pi / 180.0))
        up = matrix(math.cos(float(j + 1) * math.pi / 180.0))
        scatter[j, :, :] = (((lo + up) / 2.0) / norm)[:, None]
    return opacity, scatter


def expand_six_elements(scatter6: np.ndarray) -> np.ndarray:
    """6 -> 16 element expansion of ``atmosphere.py:42-58`` (Mie output format)."""
    n180, _, nwav = scatter6.shape
    s = np.zeros((n180, 16, nwav))
    s[:, 0] = scatter6[:, 0]
    s[:, 1] = scatter6[:, 1]
    s[:, 4] = scatter6[:, 1]
    s[:, 5] = scatter6[:, 2]
    s[:, 10] = scatter6[:, 3]
    s[:, 11] = scatter6[:, 4]
    s[:, 14] = -scatter6[:, 4]
    s[:, 15] = scatter6[:, 5]
    return s


def normalize_matrix(scatter: np.ndarray, normalizer: str = "simps") -> np.ndarray:
    """``atmosphere.py:29-65``: per wavelength divide by 2 pi simps(P11 sin(theta), theta).

    ``normalizer="simps"`` is the reference's (pre-1.11 SciPy) rule; ``"simpson"`` uses the
    installed ``scipy.integrate.simpson`` -- what the survey's probe inputs were built with
    (tests/golden/README.md), kept so the frozen reference runs can be re-driven exactly."""
    angle = np.array([(float(i) + 0.5) * math.pi / 180.0 for i in range(180)])
    out = np.array(scatter, dtype=np.float64, copy=True)
    for j in range(out.shape[2]):
        if normalizer == "simpson":
            from scipy.integrate import simpson
            norm = float(simpson(out[:, 0, j] * np.sin(angle), x=angle))
        else:
            norm = simps_avg(out[:, 0, j] * np.sin(angle), angle)
        norm *= 2.0 * math.pi
        out[:, :, j] /= norm
    return out


def write_opacity_fits(path: str, opacity: np.ndarray, scatter: np.ndarray) -> None:
    fitsio.write(path, [np.asarray(opacity, dtype=np.float64), np.asarray(scatter, dtype=np.float64)],
                 names=["", "SCATTERMATRIX"])


def read_opacity_fits(path: str):
    hdus = fitsio.read(path)
    return np.array(hdus[0].data, dtype=np.float64), np.array(hdus[1].data, dtype=np.float64)

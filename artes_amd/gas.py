"""Gas opacities and pressure-temperature profiles: Python 3 restatements of the
reference's input generators ``python/opacityGas.py``, ``python/opacityMolecules.py``,
``python/pressureTemperatureIsothermal.py`` and ``python/pressureTemperatureSelfLuminous.py``.

They write what ``atmosphere.py`` (``artes_amd.atmosphere``) consumes: opacity FITS
files (HDU 0 = [wavelength um, extinction, absorption, scattering] in cm2 g-1, HDU 1 =
the [180][16][nwav] scattering matrix) and ``pressureTemperature.dat``.  The reference
scripts are configured by editing module constants; here the same values are keyword
arguments with the reference's defaults.  Line numbers below refer to those scripts.
"""

from __future__ import annotations

import math
import os

import numpy as np
from scipy.integrate import quad

from .opacity import write_opacity_fits

AVOGADRO = 6.02214129e23     # [mol-1]
LOSCHMIDT = 2.6867805e19     # [cm-3]


def _h2_refractive_index(wavelength_um: float) -> float:
    """H2 refractive index (opacityGas.py:83-86, opacityMolecules.py:210-216)."""
    a = 13.58e-5
    b = 7.52e-3
    return 1.0 + a + a * b / (wavelength_um * wavelength_um)


def rayleigh_matrix_table(depolarization: float, nwav: int) -> np.ndarray:
    """Bin-edge-averaged depolarised Rayleigh matrix over 2 pi int P11 sin (opacityGas.py:106-150)."""
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
    scatter = np.zeros((180, 16, nwav))
    for j in range(180):
        lo = matrix(math.cos(float(j) * math.pi / 180.0))
        up = matrix(math.cos(float(j + 1) * math.pi / 180.0))
        scatter[j, :, :] = (((lo + up) / 2.0) / norm)[:, None]
    return scatter


def gas_opacity(absorption_file: str, vmr: float = 1.8e-3, mmw_abs: float = 16.04, mmw_scat: float = 2.02,
                depolarization: float = 0.02, wavelength_min: float = 0.4, wavelength_max: float = 1.0,
                absorption_wavelength: bool = False, manual_step: float = 0.001):
    """``opacityGas.py``: one absorbing molecule (absorption coefficients [cm2 molecule-1]
    per wavelength [um]) with volume mixing ratio ``vmr`` in an H2 Rayleigh-scattering gas.
    Returns (opacity [4][nwav] in cm2 g-1, scatter [180][16][nwav])."""
    w, a = np.loadtxt(absorption_file, unpack=True)
    gas_mass_abs = mmw_abs / AVOGADRO
    gas_mass_scat = mmw_scat / AVOGADRO
    a = a / gas_mass_abs                                   # [cm2 molecule-1] -> [cm2 g-1] (45)
    wavelength, absorption = [], []
    if absorption_wavelength:                              # opacityGas.py:56-63
        for i in range(len(w)):
            if w[i] >= wavelength_min:
                wavelength.append(w[i])
                absorption.append(a[i])
            if w[i] > wavelength_max:
                break
    else:                                                  # manual wavelength steps (65-73)
        wl = wavelength_min
        for i in range(len(w)):
            if w[i] >= wl and w[i] < wl + manual_step:
                wavelength.append(w[i])
                absorption.append(a[i])
                wl += manual_step
            if w[i] > wavelength_max:
                break
    opacity = np.zeros((4, len(wavelength)))
    for i, lam in enumerate(wavelength):                   # opacityGas.py:75-104
        ri = _h2_refractive_index(lam)
        dep = (6.0 + 3.0 * depolarization) / (6.0 - 7.0 * depolarization)
        rindex = ((ri * ri - 1.0) / LOSCHMIDT) ** 2.0
        cross = (8.0 * math.pi ** 3.0 / 3.0) * rindex * dep
        cross /= (lam * 1.0e-4) ** 4.0
        opacity[0, i] = lam
        opacity[1, i] = cross / gas_mass_scat + absorption[i] * vmr
        opacity[2, i] = absorption[i] * vmr
        opacity[3, i] = cross / gas_mass_scat
    return opacity, rayleigh_matrix_table(depolarization, len(wavelength))


# --------------------------------------------------------------- molecules ---
def read_pt_grid(dat_dir: str) -> np.ndarray:
    """``PTgrid.dat`` rows: file number, pressure [bar], temperature [K] (opacityMolecules.py:60)."""
    return np.genfromtxt(os.path.join(dat_dir, "PTgrid.dat"), skip_header=1)


def read_grid_opacity(dat_dir: str, filenumber: int):
    """``opacity_aver_NNNN.dat``: wavelength [um], opacity [cm2 molecule-1] (opacityMolecules.py:37-45)."""
    return np.loadtxt(os.path.join(dat_dir, "opacity_aver_" + str(int(filenumber)).zfill(4) + ".dat"), unpack=True)


def pt_corners(grid: np.ndarray, log_pressure_layer: float, temp_layer: float) -> list[int]:
    """``getPT`` (opacityMolecules.py:47-120): indices of the four PTgrid rows around a layer,
    [upper P upper T, lower P upper T, upper P lower T, lower P lower T], with the
    reference's edge rules (clamping above the grid, [0, 0, 0, 0] if a corner is missing)."""
    pressure_layer = 10.0 ** log_pressure_layer
    index_opac, p_opac, t_opac = grid[:, 0], grid[:, 1], grid[:, 2]
    n = len(index_opac)
    upper_t = lower_t = None
    for i in range(n):
        if t_opac[i] == temp_layer:
            upper_t = lower_t = t_opac[i]
            break
        elif t_opac[i] > temp_layer:
            upper_t, lower_t = t_opac[i], t_opac[i - 1]
            break
        elif t_opac[n - 1] < temp_layer:
            upper_t, lower_t = t_opac[n - 1], t_opac[n - 2]
            break
    if pressure_layer > np.max(p_opac):                    # (80-89): the last rows of each T
        uu = lu = ul = ll = None
        for i in range(n):
            if t_opac[i] == upper_t:
                uu, lu = i, i - 1
            elif t_opac[i] == lower_t:
                ul, ll = i, i - 1
        return [uu, lu, ul, ll]
    uu = lu = ul = ll = None
    for i in range(n):
        if t_opac[i] == upper_t:
            if p_opac[i] == pressure_layer:
                uu = lu = i
                break
            elif p_opac[i] > pressure_layer:
                uu, lu = i, i - 1
                break
    for i in range(n):
        if t_opac[i] == lower_t:
            if p_opac[i] == pressure_layer:
                ul = ll = i
                break
            elif p_opac[i] > pressure_layer:
                ul, ll = i, i - 1
                break
    if None in (uu, lu, ul, ll):                           # UnboundLocalError branch (118-119)
        return [0, 0, 0, 0]
    return [uu, lu, ul, ll]


def interpolate_pt(grid: np.ndarray, pressure_layer: float, temp_layer: float, idx: list[int],
                   opacity_array) -> np.ndarray:
    """``interpolateOpacityFiles`` (opacityMolecules.py:121-166): bilinear interpolation in
    log10 P, log10 T of log10 opacity (floored at -500)."""
    p1, p2 = grid[idx[1]][1], grid[idx[0]][1]
    t1, t2 = grid[idx[2]][2], grid[idx[0]][2]
    if grid[idx[3]][1] != p1 or grid[idx[2]][1] != p2 or grid[idx[3]][2] != t1 or grid[idx[1]][2] != t2:
        raise ValueError("bilinear interpolation doesn't have a square grid in interpolateOpacityFiles!")
    p1, p2, t1, t2 = np.log10(p1), np.log10(p2), np.log10(t1), np.log10(t2)
    with np.errstate(divide="ignore"):
        op = np.log10(np.asarray(opacity_array, dtype=np.float64))
    tl = np.log10(temp_layer)
    pl = np.log10(pressure_layer)
    op[op < -500] = -500
    if p1 == p2 and t1 == t2:
        return 10.0 ** op[0]
    elif p1 == p2:
        return 10.0 ** (op[2] + (op[0] - op[2]) * (tl - t1) / (t2 - t1))
    elif t1 == t2:
        return 10.0 ** (op[1] + (op[0] - op[1]) * (pl - p1) / (p2 - p1))
    r1 = ((p2 - pl) / (p2 - p1)) * op[3] + ((pl - p1) / (p2 - p1)) * op[2]
    r2 = ((p2 - pl) / (p2 - p1)) * op[1] + ((pl - p1) / (p2 - p1)) * op[0]
    return 10.0 ** (((t2 - tl) / (t2 - t1)) * r1 + ((tl - t1) / (t2 - t1)) * r2)


def molecule_opacities(pressure, temperature, dat_dir: str, wavelength_min: float = 1.6,
                       wavelength_max: float = 1.6, mmw: float = 2.02, depolarization: float = 0.0):
    """``opacityMolecules.py``: per pressure-temperature layer, the P-T interpolated molecular
    absorption and H2 Rayleigh scattering.  Returns {layer number: (opacity, scatter)}
    with the reference's numbering ``len(P) - i`` (file ``gas_opacity_NN.fits``)."""
    grid = read_pt_grid(dat_dir)
    plog = np.log10(np.asarray(pressure, dtype=np.float64))
    mass = mmw / AVOGADRO
    out = {}
    for i in range(len(plog)):                             # opacityMolecules.py:170-198
        idx = pt_corners(grid, plog[i], float(temperature[i]))
        wavelength, _ = read_grid_opacity(dat_dir, idx[0] + 1)
        ops = [read_grid_opacity(dat_dir, k + 1)[1] for k in idx]
        absorption = interpolate_pt(grid, float(pressure[i]), float(temperature[i]), idx, ops)
        absorption = absorption / mass                     # [cm2 molecule-1] -> [cm2 g-1] (254)
        rows = []
        for k in range(len(wavelength)):                   # (266-287)
            if wavelength[k] >= wavelength_min:
                ri = _h2_refractive_index(wavelength[k])
                rindex = (ri * ri - 1.0) * (ri * ri - 1.0) / ((ri * ri + 2.0) * (ri * ri + 2.0))
                dep = (6.0 + 3.0 * depolarization) / (6.0 - 7.0 * depolarization)
                cross = 24.0 * math.pi * math.pi * math.pi * rindex * dep / (((wavelength[k] * 1.0e-4) ** 4) * (LOSCHMIDT ** 2))
                rows.append((wavelength[k], cross / mass + absorption[k], absorption[k], cross / mass))
                if wavelength[k] > wavelength_max:
                    break
        opacity = np.array(rows, dtype=np.float64).T.reshape(4, len(rows))
        out[len(plog) - i] = (opacity, rayleigh_matrix_table(depolarization, len(rows)))
    return out


def write_molecule_opacities(directory: str, pressure, temperature, dat_dir: str, **kw) -> list[str]:
    """Write ``input/<atm>/opacity/gas_opacity_NN.fits`` as opacityMolecules.py does (291-300)."""
    opdir = os.path.join(directory, "opacity")
    os.makedirs(opdir, exist_ok=True)
    paths = []
    for layer, (opacity, scatter) in sorted(molecule_opacities(pressure, temperature, dat_dir, **kw).items()):
        path = os.path.join(opdir, "gas_opacity_%02d.fits" % layer)
        write_opacity_fits(path, opacity, scatter)
        paths.append(path)
    return paths


# ------------------------------------------------------- P-T profiles ---
def pt_isothermal(t_iso: float = 800.0, p_min: float = 1e-3, p_max: float = 1e2, levels: int = 40):
    """``pressureTemperatureIsothermal.py``: log-spaced pressures [bar], constant T [K]."""
    p = np.logspace(np.log10(p_min), np.log10(p_max), levels) * 1e6 * 1e-6
    return p, np.full(p.size, float(t_iso))


def pt_self_luminous(t_eff: float = 800.0, kappa: float = 1e-2, log_g: float = 3.4, p_min: float = 1e-3,
                     p_max: float = 1e2, levels: int = 20):
    """``pressureTemperatureSelfLuminous.py``: grey Eddington profile
    T = (3 Teff^4 / 4 (2/3 + tau))^(1/4), tau = kappa P / g (P in Ba, g in cm s-2)."""
    g = 10.0 ** log_g
    p = np.logspace(np.log10(p_min), np.log10(p_max), levels) * 1e6
    tau = kappa * p / g
    t = ((3.0 * (t_eff ** 4) / 4.0) * ((2.0 / 3.0) + tau)) ** (1.0 / 4.0)
    return p * 1e-6, t


def write_pt_file(directory: str, pressure, temperature) -> str:
    """``pressureTemperature.dat`` as the reference writes it (header + two columns)."""
    path = os.path.join(directory, "pressureTemperature.dat")
    os.makedirs(directory, exist_ok=True)
    with open(path, "w") as f:
        f.write("# Pressure [bar] - Temperature [K]\n\n")
        np.savetxt(f, np.column_stack([pressure, temperature]))
    return path

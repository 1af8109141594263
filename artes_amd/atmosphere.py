"""Atmosphere builder: Python 3 restatement of the reference's ``python/atmosphere.py``.

``python -m artes_amd.atmosphere <atm>`` turns ``input/<atm>/atmosphere.in`` plus the
opacity FITS files in ``input/<atm>/opacity/`` into ``input/<atm>/atmosphere.fits``
with the nine HDUs ARTES reads by position (``atmosphere.py:449-460``):
radial [m], polar [deg], azimuthal [deg], wavelength [micron], density [kg m-3],
temperature [K], scattering [m-1], absorption [m-1], scattermatrix.

Behaviour restated (``atmosphere.py`` line numbers):
* every ``opacity/*.fits`` is expanded 6 -> 16 elements if needed and renormalised
  in place with ``simps`` (``29-87``);
* the radial grid comes from ``[grid] radial`` or, with ``pressureTemperature.dat``,
  from hydrostatic scale heights (``127-167``);
* ``fitsNN`` opacities in cm2 g-1 are divided by 10 to m2 kg-1 (``240-276``);
* ``opacityNN`` regions add kappa*rho per cell and mix matrices by extinction
  weight (``330-369``); the density bookkeeping keeps the reference's indexing by
  species number (``371-377``);
* ring cells are appended beyond the outer radius (``406-445``).
"""

from __future__ import annotations

import configparser
import math
import os
import sys

import numpy as np

from . import fitsio
from .opacity import expand_six_elements, normalize_matrix

R_JUP = 69911e3
GAS_CONSTANT = 8.3144621


def normalize_opacity_dir(opacity_dir: str) -> None:
    """``atmosphere.py:29-87``: rewrite each opacity FITS with a 16-element, normalised matrix."""
    if not os.path.isdir(opacity_dir):
        return
    for name in sorted(os.listdir(opacity_dir)):
        if not name.endswith(".fits"):
            continue
        path = os.path.join(opacity_dir, name)
        hdus = fitsio.read(path)
        opacity = np.array(hdus[0].data, dtype=np.float64)
        scatter = np.array(hdus[1].data, dtype=np.float64)
        if scatter.shape[1] == 6:
            scatter = expand_six_elements(scatter)
        scatter = normalize_matrix(scatter)
        fitsio.write(path, [opacity, scatter], names=["OPACITY", "SCATTERMATRIX"])


def _split(value: str) -> list[str]:
    return [chunk.strip() for chunk in value.split(",")]


def build(directory: str, write: bool = True, normalize: bool = True) -> dict:
    """Build the atmosphere arrays for ``directory`` (= ``input/<atm>/``)."""
    directory = os.path.join(directory, "")
    opacity_dir = directory + "opacity/"
    if normalize:
        normalize_opacity_dir(opacity_dir)

    if not os.path.isfile(directory + "atmosphere.in"):
        raise FileNotFoundError(f"The atmosphere.in file does not exist in {directory}!")
    parser = configparser.ConfigParser(inline_comment_prefixes=None)
    parser.read(directory + "atmosphere.in")

    r_planet = float(parser.get("grid", "radius")) * R_JUP
    ring = parser.has_option("composition", "ring") and parser.get("composition", "ring").strip() != ""
    gas = parser.getboolean("composition", "gas", fallback=False)

    pt_file = directory + "pressureTemperature.dat"
    density_gas = np.zeros(0)
    temperature = np.zeros(0)
    pressure = scale_height = radial_gas = None
    if os.path.isfile(pt_file):
        mmw = float(parser.get("composition", "molweight")) * 1.0e-3
        log_g = float(parser.get("composition", "log_g"))
        gravity = 1e-2 * 10.0 ** log_g
        pressure, temperature = np.loadtxt(pt_file, unpack=True)
        pressure = pressure * 1.0e5
        pressure = pressure[::-1]
        temperature = temperature[::-1]
        n = len(pressure)
        scale_height = np.zeros(n)
        density_gas = np.zeros(n)
        radial = np.zeros(n)
        scale_height[0] = GAS_CONSTANT * temperature[0] / (mmw * gravity)
        density_gas[0] = pressure[0] / (gravity * scale_height[0])
        for i in range(1, n):
            scale_height[i] = GAS_CONSTANT * temperature[i] / (mmw * gravity)
            density_gas[i] = pressure[i] / (gravity * scale_height[i])
            radial[i] = radial[i - 1] - scale_height[i] * np.log(pressure[i] / pressure[i - 1])
        nr = len(radial)
        pressure = pressure[:-1]
        temperature = temperature[:-1]
        scale_height = scale_height[:-1]
        density_gas = density_gas[:-1]
        radial_gas = radial[:-1]
        radial = list(radial)
    else:
        rr = _split(parser.get("grid", "radial"))
        nr = len(rr) + 1
        radial = [0.0]
        if nr > 0 and len(rr[0]) > 0:
            for i in range(nr - 1):
                radial.append(float(rr[i]) * 1.0e3)
    radial = [r + r_planet for r in radial]

    tt = _split(parser.get("grid", "theta"))
    ntheta = 2 if not tt[0] else len(tt) + 2
    theta = [0.0] + ([float(t) for t in tt] if tt and tt[0] else []) + [180.0]

    pp = _split(parser.get("grid", "phi"))
    nphi = 1 if not pp[0] else len(pp) + 1
    phi = [0.0] + ([float(p) for p in pp] if pp and pp[0] else [])

    wavelengths = None
    n_wavelength = 0
    opacity_gas = scatter_gas = None
    if gas:
        first = fitsio.read(opacity_dir + "gas_opacity_01.fits")
        n_wavelength = first[0].data.shape[1]
        wavelengths = np.array(first[0].data[0], dtype=np.float64)
        opacity_gas = np.zeros((density_gas.size, 4, n_wavelength))
        scatter_gas = np.zeros((density_gas.size, 180, 16, n_wavelength))
        for i in range(density_gas.size):
            h = fitsio.read(opacity_dir + f"gas_opacity_{i + 1:02d}.fits")
            opacity_gas[i] = h[0].data / 10.0
            scatter_gas[i] = h[1].data

    n_other = 0
    while parser.has_option("composition", f"fits{n_other + 1:02d}"):
        n_other += 1
    opacity_other = scatter_other = None
    if n_other > 0:
        first = fitsio.read(opacity_dir + parser.get("composition", "fits01").strip())
        n_wavelength = first[0].data.shape[1]
        wavelengths = np.array(first[0].data[0], dtype=np.float64)
        opacity_other = np.zeros((n_other, 4, n_wavelength))
        scatter_other = np.zeros((n_other, 180, 16, n_wavelength))
        for i in range(n_other):
            h = fitsio.read(opacity_dir + parser.get("composition", f"fits{i + 1:02d}").strip())
            opacity_other[i] = h[0].data / 10.0
            scatter_other[i] = h[1].data
    if wavelengths is None:
        raise ValueError("no opacity source (gas or fitsNN) defined in atmosphere.in")

    composition, r_in, r_out, t_in, t_out, p_in, p_out, density_other = [], [], [], [], [], [], [], []
    i = 1
    while parser.has_option("composition", f"opacity{i:02d}"):
        aa = _split(parser.get("composition", f"opacity{i:02d}"))
        if "nr" in aa[3]:
            aa[3] = nr - 1
        if "ntheta" in str(aa[5]):
            aa[5] = ntheta - 1
        if "nphi" in str(aa[7]):
            aa[7] = nphi
        composition.append(int(aa[0]))
        r_in.append(int(aa[2]))
        r_out.append(int(aa[3]))
        t_in.append(int(aa[4]))
        t_out.append(int(aa[5]))
        p_in.append(int(aa[6]))
        p_out.append(int(aa[7]))
        try:
            density_other.append(float(aa[1]) * 1e3)
        except ValueError:
            pass
        i += 1

    k_sca = np.zeros((n_wavelength, nphi, ntheta - 1, nr - 1))
    k_abs = np.zeros((n_wavelength, nphi, ntheta - 1, nr - 1))
    scatter = np.zeros((180, 16, n_wavelength, nphi, ntheta - 1, nr - 1))
    density = np.zeros((nphi, ntheta - 1, nr - 1))

    if gas:
        for ir in range(nr - 1):
            for m in range(n_wavelength):
                k_abs[m, :, :, ir] = density_gas[ir] * opacity_gas[ir, 2, m]
                k_sca[m, :, :, ir] = density_gas[ir] * opacity_gas[ir, 3, m]
                scatter[:, :, m, :, :, ir] = scatter_gas[ir, :, :, m][:, :, None, None]
        for ir in range(nr - 1):
            density[:, :, ir] = density_gas[ir]

    for n in range(len(composition)):
        c = composition[n] - 1
        for m in range(n_wavelength):
            o_sca = density_other[n] * opacity_other[c, 3, m]
            o_abs = density_other[n] * opacity_other[c, 2, m]
            for k in range(p_in[n], p_out[n]):
                for j in range(t_in[n], t_out[n]):
                    for ir in range(r_in[n], r_out[n]):
                        if density[k, j, ir] == 0.0:
                            scatter[:, :, m, k, j, ir] = scatter_other[c, :, :, m]
                        elif density[k, j, ir] > 0.0:
                            w = (o_sca + o_abs) / (o_sca + o_abs + k_sca[m, k, j, ir] + k_abs[m, k, j, ir])
                            scatter[:, :, m, k, j, ir] *= (1.0 - w)
                            scatter[:, :, m, k, j, ir] += w * scatter_other[c, :, :, m]
                        k_sca[m, k, j, ir] += o_sca
                        k_abs[m, k, j, ir] += o_abs
    for n in range(len(composition)):
        # reference quirk (atmosphere.py:371-377): indexed by species number, not by entry
        dens = density_other[composition[n] - 1]
        density[p_in[n]:p_out[n], t_in[n]:t_out[n], r_in[n]:r_out[n]] += dens

    temperature_grid = np.zeros((nphi, ntheta - 1, nr - 1))
    if os.path.isfile(pt_file):
        temperature_grid[:, :, :] = temperature[None, None, : nr - 1]
        if write:
            z = np.column_stack([pressure * 1.0e-5, temperature, density_gas * 1.0e-3,
                                 scale_height * 1.0e-3, radial_gas * 1.0e-3])
            with open(directory + "atmosphere.dat", "w") as f:
                f.write("# Pressure [bar] - Temperature [K] - Gas density [g/cm3] - Scale Height [km] - Altitude [km] \n\n")
                np.savetxt(f, z)

    radial = np.array(radial, dtype=np.float64)
    if ring:
        aa = _split(parser.get("composition", "ring"))
        r_max = np.amax(radial)
        radial = np.append(radial, [r_max + float(aa[3]) * 1e3, r_max + float(aa[4]) * 1e3])
        t0, t1 = int(aa[5]), int(aa[6])
        rd = np.zeros((nphi, ntheta - 1, 2))
        rd[:, t0:t1, 1] = float(aa[1])
        density = np.append(density, rd, axis=2)
        rt = np.zeros((nphi, ntheta - 1, 2))
        rt[:, t0:t1, 1] = float(aa[2])
        temperature_grid = np.append(temperature_grid, rt, axis=2)
        rs = np.zeros((n_wavelength, nphi, ntheta - 1, 2))
        ra = np.zeros((n_wavelength, nphi, ntheta - 1, 2))
        rm = np.zeros((180, 16, n_wavelength, nphi, ntheta - 1, 2))
        sp = int(aa[0]) - 1
        for m in range(n_wavelength):
            rs[m, :, t0:t1, 1] = float(aa[1]) * opacity_other[sp, 3, m]
            ra[m, :, t0:t1, 1] = float(aa[1]) * opacity_other[sp, 2, m]
            rm[:, :, m, :, t0:t1, 1] = scatter_other[sp, :, :, m][:, :, None, None]
        k_sca = np.append(k_sca, rs, axis=3)
        k_abs = np.append(k_abs, ra, axis=3)
        scatter = np.append(scatter, rm, axis=5)

    atm = dict(radial=radial, theta=np.array(theta, dtype=np.float64), phi=np.array(phi, dtype=np.float64),
               wavelength=np.asarray(wavelengths, dtype=np.float64), density=density,
               temperature=temperature_grid, scattering=k_sca, absorption=k_abs, scattermatrix=scatter)
    if write:
        write_atmosphere_fits(directory + "atmosphere.fits", atm)
    return atm


HDU_ORDER = ("radial", "theta", "phi", "wavelength", "density", "temperature",
             "scattering", "absorption", "scattermatrix")
HDU_NAMES = ("RADIAL", "POLAR", "AZIMUTHAL", "WAVELENGTH", "DENSITY", "TEMPERATURE",
             "SCATTERING", "ABSORPTION", "SCATTERMATRIX")


def write_atmosphere_fits(path: str, atm: dict) -> None:
    fitsio.write(path, [np.asarray(atm[k], dtype=np.float64) for k in HDU_ORDER], names=HDU_NAMES)


def read_atmosphere_fits(path: str) -> dict:
    """Positional read of the nine HDUs, as ``get_atmosphere`` does (``ARTES.f90:2067-2198``)."""
    hdus = fitsio.read(path)
    if len(hdus) < 9:
        raise ValueError(f"{path}: expected 9 HDUs, found {len(hdus)}")
    return {k: np.asarray(hdus[i].data, dtype=np.float64) for i, k in enumerate(HDU_ORDER)}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("usage: python -m artes_amd.atmosphere <atmosphere> [root]")
        return 1
    root = argv[1] if len(argv) > 1 else os.getcwd()
    build(os.path.join(root, "input", argv[0]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""Host-side restatement of the reference's run driver around the transport kernel.

Everything here is O(pixels) or O(cells) bookkeeping; the O(packets) work goes to
the HIP engine (``artes_amd.engine``).  Reference routines restated:

* detector geometry of ``initialize``          ``ARTES.f90:451-514``
* ``planck_function``                           ``ARTES.f90:1350-1367``
* ``photon_package``                            ``ARTES.f90:2509-2539``
* thread reduction + photometry                 ``ARTES.f90:957-1004``
* ``write_output`` (stokes/error/photometry/...) ``ARTES.f90:3472-3772``
* the run-mode loop ``run``                     ``ARTES.f90:121-267``
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

from . import fitsio
from .config import CC, HH, K_B, PI, RunConfig


@dataclass
class Detector:
    """Detector geometry derived in ``initialize`` (``ARTES.f90:453-514``)."""

    nx: int
    ny: int
    det_theta: float
    det_phi: float
    x_max: float
    y_max: float
    x_fov: float
    y_fov: float
    pixel_scale: float
    phase_observer: float


def spherical_cartesian(r, theta, phi):
    """``ARTES.f90:1421-1432``."""
    return r * math.sin(theta) * math.cos(phi), r * math.sin(theta) * math.sin(phi), r * math.cos(theta)


def detector_geometry(cfg: RunConfig, r_top: float) -> Detector:
    nx, ny = cfg.nx, cfg.ny
    det_theta, det_phi = cfg.det_theta, cfg.det_phi
    if cfg.spectrum:
        nx = ny = 1
    elif cfg.phase_curve:
        nx = ny = 1
        det_theta = PI / 2.0
        det_phi = 1.0e-5
    x_max = 1.3 * r_top * (cfg.oblateness + 1.0)
    y_max = 1.3 * r_top * (cfg.oblateness + 1.0)
    x_fov = 2.0 * math.atan(x_max / cfg.distance_planet) * 3600.0 * 180.0 / PI * 1000.0
    y_fov = 2.0 * math.atan(y_max / cfg.distance_planet) * 3600.0 * 180.0 / PI * 1000.0
    pixel_scale = x_fov / nx
    if abs(det_phi) < 1.0e-3 or det_phi > 2.0 * PI - 1.0e-3:
        det_phi = 1.0e-3
    if PI - 1.0e-3 < det_phi < PI + 1.0e-3:
        det_phi = PI - 1.0e-3
    phase_obs = 0.0
    if not cfg.phase_curve:
        c = (math.sin(cfg.theta_star) * math.cos(cfg.phi_star) * math.sin(det_theta) * math.cos(det_phi)
             + math.sin(cfg.theta_star) * math.sin(cfg.phi_star) * math.sin(det_theta) * math.sin(det_phi)
             + math.cos(cfg.theta_star) * math.cos(det_theta))
        phase_obs = math.acos(max(-1.0, min(1.0, c))) * 180.0 / PI
    return Detector(nx, ny, det_theta, det_phi, x_max, y_max, x_fov, y_fov, pixel_scale, phase_obs)


PHASE_ANGLES_DEG = None  # computed by phase_angles()


def phase_angles() -> list[float]:
    """The 73 detector azimuths of the phase-curve loop (``ARTES.f90:215-230``), in radians."""
    out = []
    det_phi = 0.0
    for i in range(1, 74):
        if i == 1:
            det_phi = 1.0e-5 * PI / 180.0
        elif i == 2:
            det_phi = 2.5 * PI / 180.0
        elif i == 73:
            det_phi = (180.0 - 1e-5) * PI / 180.0
        else:
            det_phi = det_phi + 2.5 * PI / 180.0
        out.append(det_phi)
    return out


def planck(temperature: float, wavelength_m: float, photon_source: int) -> float:
    """``planck_function`` (``ARTES.f90:1350-1367``)."""
    x = HH * CC / (wavelength_m * K_B * temperature)
    if photon_source == 1:
        return (2.0 * PI * HH * CC * CC / (wavelength_m ** 5.0)) / math.expm1(x) if x < 700 else 0.0
    return (2.0 * HH * CC * CC / (wavelength_m ** 5.0)) / math.expm1(x) if x < 700 else 0.0


def package_energy(cfg: RunConfig, wavelength_m: float, r_top: float, packages: int, det_phi: float,
                   emissivity_total: float | None = None) -> float:
    """``photon_package`` (``ARTES.f90:2509-2539``).  The planet source needs the total weighted
    emissivity of the wavelength (``Grid.thermal``)."""
    if cfg.photon_source == 2:
        if emissivity_total is None:
            raise ValueError("photon:source=planet: package_energy needs the emissivity total")
        return emissivity_total / (cfg.distance_planet * cfg.distance_planet * float(packages))
    flux = planck(cfg.t_star, wavelength_m, 1)
    e = PI * flux * r_top * r_top * cfg.r_star * cfg.r_star / (
        cfg.orbit * cfg.orbit * cfg.distance_planet * cfg.distance_planet * float(packages))
    if cfg.phase_curve and det_phi * 180.0 / PI >= 170.0:
        e = e * (PI * cfg.r_star ** 2 - 0.9 * 0.9 * PI * cfg.r_star ** 2) / (PI * cfg.r_star ** 2)
    return e


def scale_detector(raw: np.ndarray, energy: float) -> np.ndarray:
    """Per-thread sums -> detector (``ARTES.f90:959-975``). raw/out shape [3][4][ny][nx]."""
    det = np.array(raw, dtype=np.float64, copy=True)
    det[0] *= energy
    det[1] *= energy * energy
    return det


def photometry(det: np.ndarray) -> np.ndarray:
    """``photometry(1:11)`` (``ARTES.f90:977-1004``); returned 0-based (index k <-> photometry(k+1))."""
    ph = np.zeros(11)
    ph[0] = det[0, 0].sum()
    ph[2] = det[0, 1].sum()
    ph[4] = det[0, 2].sum()
    ph[6] = det[0, 3].sum()
    ph[8] = math.sqrt(det[0, 1].sum() ** 2 + det[0, 2].sum() ** 2)
    ph[9] = ph[8] / ph[0] if ph[0] != 0 else float("nan")
    for i in range(4):
        n = det[2, i].sum()
        if n > 0.0:
            dummy = det[1, i].sum() / n - (det[0, i].sum() / n) ** 2
            if dummy > 0.0:
                ph[2 * i + 1] = math.sqrt(dummy) * math.sqrt(n)
    if ph[2] ** 2 + ph[4] ** 2 > 0.0:
        dpi = math.sqrt(((ph[2] * ph[3]) ** 2 + (ph[4] * ph[5]) ** 2) / (2.0 * (ph[2] ** 2 + ph[4] ** 2)))
        ph[10] = ph[9] * math.sqrt((dpi / ph[8]) ** 2 + (ph[1] / ph[0]) ** 2)
    return ph


def error_image(det: np.ndarray) -> np.ndarray:
    """Per-pixel sigma and polarisation error (``ARTES.f90:3483-3519``); shape [5][ny][nx].

    Plane 5 keeps the reference's use of ``pol``/``dpol`` carried over from the
    previous pixel when a pixel has Q=U=0 (``ARTES.f90:3506-3516``); it is not a
    parity quantity."""
    _, _, ny, nx = det.shape
    err = np.zeros((5, ny, nx))
    with np.errstate(divide="ignore", invalid="ignore"):
        for k in range(4):
            n = det[2, k]
            dummy = np.where(n > 0, det[1, k] / np.where(n > 0, n, 1) - (det[0, k] / np.where(n > 0, n, 1)) ** 2, 0.0)
            err[k] = np.where((n > 0) & (dummy > 0), np.sqrt(np.clip(dummy, 0, None)) * np.sqrt(n), 0.0)
        pol = 0.0
        dpol = 0.0
        for j in range(ny):          # Fortran loop order: i (x) fastest
            for i in range(nx):
                q, u = det[0, 1, j, i], det[0, 2, j, i]
                if q * q + u * u > 0.0:
                    pol = math.sqrt(q * q + u * u)
                    dpol = math.sqrt(((q * err[1, j, i]) ** 2 + (u * err[2, j, i]) ** 2) / (2.0 * (q * q + u * u)))
                ii = det[0, 0, j, i]
                if ii > 0.0:
                    a = pol / ii
                    b = (dpol / pol) ** 2 if pol != 0 else float("nan")
                    err[4, j, i] = a * math.sqrt(b + (err[0, j, i] / ii) ** 2) if not math.isnan(b) else float("nan")
    return err


def _fmt(x: float) -> str:
    return f"{x:.17G}"


def write_stokes_outputs(outdir: str, det: np.ndarray, pixel_scale: float) -> None:
    """``write_fits_3D`` calls of ``write_output`` (``ARTES.f90:3569-3570``)."""
    os.makedirs(outdir, exist_ok=True)
    fitsio.write(os.path.join(outdir, "stokes.fits"), det[0] * 1.0e-6 / (pixel_scale * pixel_scale))
    fitsio.write(os.path.join(outdir, "error.fits"), error_image(det))


def write_photometry(outdir: str, wavelength_m: float, ph: np.ndarray) -> None:
    """``photometry.dat`` (``ARTES.f90:3576-3587``)."""
    with open(os.path.join(outdir, "photometry.dat"), "w") as f:
        f.write(" # Wavelength [micron] - Stokes I, Q, U, V [W m-2 micron-1]\n\n")
        vals = [wavelength_m * 1.0e6] + [1.0e-6 * ph[i] for i in range(8)]
        f.write(" " + " ".join(_fmt(v) for v in vals) + "\n")


def _append(path: str, header: str | None, line: str) -> None:
    exists = os.path.exists(path)
    with open(path, "a") as f:
        if not exists and header is not None:
            f.write(header)
        f.write(line)


def write_normalization(outdir: str, cfg: RunConfig, wavelength_m: float, r_top: float) -> None:
    """``normalization.dat`` (``ARTES.f90:3623-3652``)."""
    flux = planck(cfg.t_star, wavelength_m, 1)
    n1 = 1.0e-6 * flux * cfg.r_star ** 2 / cfg.distance_planet ** 2
    n2 = 1.0e-6 * flux * r_top ** 2 * cfg.r_star ** 2 / (cfg.orbit ** 2 * cfg.distance_planet ** 2)
    _append(os.path.join(outdir, "normalization.dat"), None,
            " " + " ".join(_fmt(v) for v in (wavelength_m * 1e6, n1, n2)) + "\n")


def write_luminosity(outdir: str, wavelength_m: float, flux_emitted: float, flux_exit: float, e_pack: float) -> None:
    """``luminosity.dat`` of the planet source (``ARTES.f90:3660-3680``): wavelength [m] (the
    reference's header says [deg]), emitted and emergent luminosity [W micron-1], and the
    emergent sum of packet weights."""
    _append(os.path.join(outdir, "luminosity.dat"),
            " # Wavelength [deg] - Emitted luminosity [W micron-1] - Emergent luminosity [W micron-1] - "
            "Emergent luminosity [a.u.]\n\n",
            " " + " ".join(_fmt(v) for v in (wavelength_m, flux_emitted * e_pack * 1.0e-6,
                                             flux_exit * e_pack * 1.0e-6, flux_exit)) + "\n")


def write_cell_luminosity(outdir: str, lum: np.ndarray) -> None:
    """``cell_luminosity.fits`` (``write_fits_3D``, ``ARTES.f90:3658``): [nphi][ntheta][nr] in C order."""
    fitsio.write(os.path.join(outdir, "cell_luminosity.fits"), np.asarray(lum, dtype=np.float64))


def flow_global_output(flow: np.ndarray, cell_depth: int) -> np.ndarray:
    """``flow_global.fits`` contents (``write_output``, ``ARTES.f90:3715-3740``): per cell at
    or above ``cell_depth`` the summed (r, theta, phi) transport vector normalised to unit
    length (left as is when zero); cells below ``cell_depth`` are zero.  [nphi][ntheta][nr][3]."""
    out = np.zeros_like(np.asarray(flow, dtype=np.float64))
    f = np.asarray(flow, dtype=np.float64)[:, :, cell_depth:, :]
    norm = np.sqrt(f[..., 0] ** 2 + f[..., 1] ** 2 + f[..., 2] ** 2)
    out[:, :, cell_depth:, :] = np.where(norm[..., None] > 0.0, f / np.where(norm > 0.0, norm, 1.0)[..., None], f)
    return out


def flow_latitudinal_output(flow: np.ndarray, cell_depth: int, flux_exit: float | None) -> np.ndarray:
    """``flow_latitudinal.fits`` contents (``ARTES.f90:3744-3766``): per cell at or above
    ``cell_depth`` the Stokes I leaving upward, downward, southward and northward, divided
    by the total emergent flux ``sum(flux_exit)``.  [nphi][ntheta][nr][4].  ``flux_exit``
    None (star source, where the reference's array is undefined): not normalised."""
    out = np.zeros_like(np.asarray(flow, dtype=np.float64))
    out[:, :, cell_depth:, :] = np.asarray(flow, dtype=np.float64)[:, :, cell_depth:, :]
    return out / flux_exit if flux_exit is not None else out


def write_flow_global(outdir: str, flow: np.ndarray, cell_depth: int) -> None:
    """``flow_global.fits`` (``write_fits_4D``, ``ARTES.f90:3738``)."""
    fitsio.write(os.path.join(outdir, "flow_global.fits"), flow_global_output(flow, cell_depth))


def write_flow_latitudinal(outdir: str, flow: np.ndarray, cell_depth: int, flux_exit: float | None) -> None:
    """``flow_latitudinal.fits`` (``write_fits_4D``, ``ARTES.f90:3766``)."""
    fitsio.write(os.path.join(outdir, "flow_latitudinal.fits"), flow_latitudinal_output(flow, cell_depth, flux_exit))


def write_cell_depth(outdir: str, wavelength_m: float, cell_depth: int) -> None:
    """``cell_depth.dat`` (``ARTES.f90:3689-3711``)."""
    _append(os.path.join(outdir, "cell_depth.dat"), " # Wavelength [micron] - Cell depth\n\n",
            f" {_fmt(wavelength_m * 1e6)} {cell_depth}\n")


def radial_optical_depths(atm: dict, wl: int) -> tuple[float, float, float]:
    """Radial optical depths of the column at theta = phi = cell 0 (``grid_initialize(2)``,
    ``ARTES.f90:2481-2485``): sum over the radial cells i = 0..nr-1, in that order, of
    (rfront(i+1) - rfront(i)) x the cell's extinction (scattering + absorption, ``2181``),
    absorption and scattering opacity.  Returns (total, absorption, scattering)."""
    rf = np.asarray(atm["radial"], dtype=np.float64)
    sca = np.asarray(atm["scattering"], dtype=np.float64)[wl, 0, 0, :]   # [nwav][nphi][ntheta][nr]
    ab = np.asarray(atm["absorption"], dtype=np.float64)[wl, 0, 0, :]
    tot = t_sca = t_abs = 0.0
    for i in range(rf.size - 1):
        dr = float(rf[i + 1] - rf[i])
        tot += dr * float(sca[i] + ab[i])
        t_sca += dr * float(sca[i])
        t_abs += dr * float(ab[i])
    return tot, t_abs, t_sca


def write_optical_depth(outdir: str, wavelength_m: float, atm: dict, wl: int) -> None:
    """``optical_depth.dat`` (``ARTES.f90:2457-2491``): appended once per wavelength in the
    ``spectrum`` and ``imaging_broad`` modes -- wavelength [micron], total, absorption and
    scattering radial optical depth."""
    tot, t_abs, t_sca = radial_optical_depths(atm, wl)
    _append(os.path.join(outdir, "optical_depth.dat"),
            " # Wavelength [micron] - Total optical depth - Absorption optical depth - Scattering optical depth\n\n",
            " " + " ".join(_fmt(v) for v in (wavelength_m * 1e6, tot, t_abs, t_sca)) + "\n")


def write_spectrum_line(outdir: str, wavelength_m: float, det: np.ndarray) -> None:
    """``spectrum.dat`` (``ARTES.f90:3591-3621``)."""
    vals = [wavelength_m * 1e6] + [1e-6 * det[0, k, 0, 0] for k in range(4)]
    _append(os.path.join(outdir, "spectrum.dat"), " # Wavelength [micron] - Stokes I, Q, U, V [W m-2 micron-1]\n\n",
            " " + " ".join(_fmt(v) for v in vals) + "\n")


def write_phase_line(outdir: str, det_phi: float, det: np.ndarray) -> None:
    """``phase.dat`` (``ARTES.f90:3521-3563``)."""
    err = error_image(det)
    deg = det_phi * 180.0 / PI
    ang = 0.0 if deg < 1.0 else (180.0 if deg > 179.0 else deg)
    vals = [ang]
    for k in range(4):
        vals += [det[0, k, 0, 0] * 1e-6, err[k, 0, 0] * 1e-6]
    _append(os.path.join(outdir, "phase.dat"), " # Wavelength [micron] - Stokes I, Q, U, V [W m-2 micron-1]\n\n",
            " " + " ".join(_fmt(v) for v in vals) + "\n")


def write_plot_dat(rundir: str, cfg: RunConfig, r_surface: float, ntheta: int, x_fov: float) -> None:
    """``python`` subroutine (``ARTES.f90:1328-1348``)."""
    with open(os.path.join(rundir, "plot.dat"), "w") as f:
        f.write("[plot]\n")
        f.write(f"photon_source={cfg.photon_source}\n")
        f.write(f"distance={cfg.distance_planet:.7E}\n")
        f.write(f"planet_radius={r_surface:.7E}\n")
        f.write(f"ntheta={ntheta}\n")
        f.write(f"fov={x_fov:.7E}\n")


def write_error_log(path: str, err_counts) -> None:
    """error.log: one ' error NNN' line per occurrence (capped at 1000 per code)."""
    with open(path, "a") as f:
        for code, n in enumerate(err_counts):
            n = int(n)
            for _ in range(min(n, 1000)):
                f.write(f" error {code:03d}\n")
            if n > 1000:
                f.write(f" error {code:03d} repeated {n} times in total\n")


def run_params(cfg: RunConfig, det: Detector, wl_index: int = 0, det_phi: float | None = None,
               cell_depth: int = -1, packet_moments: bool = True):
    """Pack the globals ``radiative_transfer`` reads into the C-ABI ``artes_run_params``.

    ``packet_moments``: also accumulate the packet-level second moments (detector planes
    12-15, totals[4:8]) that the honest-error statistics (``stats.py``) need.  The
    reference's outputs do not use them; the drop-in CLI and the bench turn them off."""
    from .abi import RunParams

    phi = det.det_phi if det_phi is None else det_phi
    return RunParams(
        wl_index=int(wl_index), nx=int(det.nx), ny=int(det.ny), photon_source=int(cfg.photon_source),
        photon_scattering=int(bool(cfg.photon_scattering)),
        phase_far=int(bool(cfg.phase_curve and phi * 180.0 / PI >= 170.0)),
        stellar_direction=int(bool(cfg.stellar_direction)), cell_depth=int(cell_depth),
        det_theta=float(det.det_theta), det_phi=float(phi), x_max=float(det.x_max), y_max=float(det.y_max),
        fstop=float(cfg.fstop), photon_minimum=float(cfg.photon_minimum), surface_albedo=float(cfg.surface_albedo),
        theta_star=float(cfg.theta_star), phi_star=float(cfg.phi_star),
        photon_emission=int(cfg.photon_emission), thermal_weight=int(bool(cfg.thermal_weight)),
        ring=int(bool(cfg.ring)), packet_moments=int(bool(packet_moments)), photon_bias=float(cfg.photon_bias))


def default_config() -> RunConfig:
    """The template ``artes.in`` used by every benchmark configuration."""
    cfg = RunConfig()
    for k, v in (("detector:type", "imaging_mono"), ("detector:theta", "90"), ("detector:phi", "90"),
                 ("detector:pixel", "25"), ("detector:distance", "10"), ("star:temperature", "5800"),
                 ("star:radius", "1"), ("planet:orbit", "5"), ("photon:fstop", "1d-5"),
                 ("photon:minimum", "1d-20")):
        cfg.apply(k, v)
    return cfg

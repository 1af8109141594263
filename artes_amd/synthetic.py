"""Synthetic atmospheres for the benchmark / parity configurations.

All share: planet radius 1 R_J (``atmosphere.py:117``), a 100 km atmosphere with
equally spaced radial faces, uniform extinction with radial optical depth ``tau``,
single-scattering albedo ``omega`` (default 1), one wavelength (0.7 micron).
The scattering matrices come from the restated opacity generators and the
``simps`` renormalisation of ``atmosphere.py:60-65``, i.e. the reference's own
setup path, not a hand-normalised table.

=========  ==============================================  ==================
config     scattering                                      grid (r x theta x phi)
=========  ==============================================  ==================
``iso``    isotropic                                       10 x 1 x 1
``hg``     Henyey-Greenstein g=0.8, pLinear 0.5            32 x 1 x 1
``ray3d``  Rayleigh, depolarisation 0                      32 x 16 x 32
=========  ==============================================  ==================
"""

from __future__ import annotations

import os

import numpy as np

from . import opacity as op
from .atmosphere import R_JUP

CONFIGS = {
    "iso": dict(kind="iso", nr=10, ntheta=1, nphi=1),
    "hg": dict(kind="hg", nr=32, ntheta=1, nphi=1, g=0.8, p_linear=0.5),
    "ray1d": dict(kind="ray", nr=32, ntheta=1, nphi=1),
    "ray3d": dict(kind="ray", nr=32, ntheta=16, nphi=32),
}


def scatter_matrix(kind: str, wavelength=(0.7,), g: float = 0.8, p_linear: float = 0.5,
                   depolarization: float = 0.0, normalizer: str = "simps") -> np.ndarray:
    wl = list(wavelength)
    if kind == "iso":
        _, s = op.isotropic(wl)
    elif kind == "hg":
        _, s = op.henyey_greenstein(wl, g1=g, w1=1.0, p_linear=p_linear, p_circular=0.0)
    elif kind == "ray":
        _, s = op.rayleigh(wl, depolarization=depolarization)
    else:
        raise ValueError(f"unknown scattering kind {kind!r}")
    return op.normalize_matrix(s, normalizer)


def make(kind: str = "ray", nr: int = 32, ntheta: int = 16, nphi: int = 32, tau: float = 1.0,
         omega: float = 1.0, height: float = 100e3, radius: float = R_JUP, wavelength=(0.7,),
         g: float = 0.8, p_linear: float = 0.5, depolarization: float = 0.0,
         share_matrix: bool = False, normalizer: str = "simps") -> dict:
    """Return the nine atmosphere arrays (same keys/layout as ``read_atmosphere_fits``).

    ``share_matrix=True`` returns the scatter matrix as a broadcast view (no 2880 x ncells
    copy); the engine deduplicates per-cell matrices anyway, so this only saves host RAM.
    """
    nwav = len(wavelength)
    radial = radius + np.linspace(0.0, height, nr + 1)
    theta = np.linspace(0.0, 180.0, ntheta + 1)
    phi = np.linspace(0.0, 360.0, nphi + 1)[:-1]
    shape = (nphi, ntheta, nr)
    kappa = tau / height
    k_ext = np.full((nwav,) + shape, kappa)
    k_sca = k_ext * omega
    k_abs = k_ext - k_sca
    sm = scatter_matrix(kind, wavelength, g=g, p_linear=p_linear, depolarization=depolarization, normalizer=normalizer)
    full = np.broadcast_to(sm[:, :, :, None, None, None], (180, 16, nwav) + shape)
    return dict(radial=radial, theta=theta, phi=phi, wavelength=np.asarray(wavelength, dtype=np.float64),
                density=np.ones(shape), temperature=np.zeros(shape), scattering=k_sca, absorption=k_abs,
                scattermatrix=full if share_matrix else np.ascontiguousarray(full))


def make_config(name: str, **over) -> dict:
    spec = dict(CONFIGS[name])
    spec.update(over)
    return make(**spec)


CLOUDY_IN = """[grid]
radius: 1.
radial:
theta: 30, 60, 90, 120, 150
phi: 60, 120, 180, 240, 300

[composition]
gas: on
molweight: 2.3
log_g: 3.4
fits01: cloud.fits
opacity01: 1, {cloud_density}, 4, 12, 1, 4, 0, 3
ring:
"""


def make_cloudy(directory: str, wavelength=(0.5, 0.7, 0.9), levels: int = 17, p_max: float = 10.0,
                cloud_density: float = 5e-13, gas_absorption: float = 0.05) -> dict:
    """BASELINE configs[3]'s input shape, scaled down: a gas atmosphere with a Mie cloud
    patch, several wavelengths, built through the reference's own setup path.

    Writes ``directory`` = ``input/<atm>/`` as a user of ``python/atmosphere.py`` would:
    an isothermal ``pressureTemperature.dat`` (``pressureTemperatureIsothermal.py``),
    one gas opacity file per layer (H2 Rayleigh from ``opacityRayleigh.py`` plus a grey
    absorption that grows with depth), a Mie cloud opacity file (``opacityMie.py``,
    restated in ``artes_amd.mie``; constant refractive index 1.5+0.001i, gamma size
    distribution r_eff 0.5 micron) and an ``atmosphere.in`` that places the cloud in
    radial layers 4-11, theta cells 1-3 and phi cells 0-2 of a 16 x 6 x 6 grid; then runs
    ``artes_amd.atmosphere.build`` (``atmosphere.py``), which writes ``atmosphere.fits``.

    The cloud is mixed into the gas by extinction weight (``atmosphere.py:366-369``), so
    every cloudy layer and wavelength has its own scattering matrix (25 distinct ones):
    more than the event kernel can stage in LDS, i.e. the per-cell matrix-id path.
    """
    from . import gas, mie

    opd = os.path.join(directory, "opacity")
    os.makedirs(opd, exist_ok=True)
    wl = [float(w) for w in wavelength]
    p, t = gas.pt_isothermal(1200.0, 1e-4, p_max, levels)
    gas.write_pt_file(directory, p, t)
    op_r, sc_r = op.rayleigh(wl)
    for i in range(levels - 1):
        o = op_r.copy()
        o[2] = o[3] * gas_absorption * (i + 1)
        o[1] = o[2] + o[3]
        op.write_opacity_fits(os.path.join(opd, f"gas_opacity_{i + 1:02d}.fits"), o, sc_r)
    ri = (np.array([0.3, 1.0]), np.array([1.5, 1.5]), np.array([1e-3, 1e-3]))
    oc, sc = mie.mie_opacity(ri, wl, density=1.0, nr=200, r_eff=0.5, v_eff=0.1)
    op.write_opacity_fits(os.path.join(opd, "cloud.fits"), oc, sc)
    with open(os.path.join(directory, "atmosphere.in"), "w") as f:
        f.write(CLOUDY_IN.format(cloud_density=cloud_density))
    from . import atmosphere

    return atmosphere.build(directory)


def make_thermal(kind: str = "ray", nr: int = 16, ntheta: int = 8, nphi: int = 8, tau_abs: float = 1.0,
                 tau_sca: float = 1.0, temperature=1000.0, height: float = 100e3, radius: float = R_JUP,
                 wavelength=(10.0,), **kw) -> dict:
    """A thermally emitting atmosphere (``photon:source=planet``): uniform absorption and
    scattering of radial optical depths ``tau_abs`` / ``tau_sca`` and a temperature that is
    either a constant or a callable of the cell-centre radius [m] (e.g. a lapse rate)."""
    atm = make(kind=kind, nr=nr, ntheta=ntheta, nphi=nphi, tau=1.0, height=height, radius=radius,
               wavelength=wavelength, **kw)
    shape = atm["temperature"].shape
    nwav = len(wavelength)
    atm["absorption"] = np.full((nwav,) + shape, tau_abs / height)
    atm["scattering"] = np.full((nwav,) + shape, tau_sca / height)
    rc = 0.5 * (atm["radial"][1:] + atm["radial"][:-1])
    t = temperature(rc) if callable(temperature) else np.full(nr, float(temperature))
    atm["temperature"] = np.broadcast_to(np.asarray(t, dtype=np.float64)[None, None, :], shape).copy()
    return atm


SELF_LUMINOUS_IN = """[grid]
radius: 1.
radial:
theta: {theta}
phi: {phi}

[composition]
gas: on
molweight: 2.02
log_g: 3.4
ring:
"""


def make_self_luminous(directory: str, fixture: str, theta: str = "30, 60, 90, 120, 150",
                       phi: str = "90, 180, 270", wavelengths=None) -> dict:
    """BASELINE configs[4]'s input: a self-luminous gas atmosphere with P-T dependent
    molecular opacities, built through the reference's setup path from a committed
    opacity fixture (``tests/golden/molecular``, made by tools/make_molecular_fixture.py
    from dat/molecules with ``artes_amd.gas.molecule_opacities``, i.e. opacityMolecules.py).

    Writes ``directory`` = ``input/<atm>/`` as the reference's scripts would:
    ``pressureTemperature.dat`` (pressureTemperatureSelfLuminous.py), one
    ``opacity/gas_opacity_NN.fits`` per P-T layer (opacity from the fixture, H2 Rayleigh
    matrices regenerated, opacityMolecules.py:291-300) and an ``atmosphere.in`` with the gas
    branch on (a ``theta`` x ``phi`` grid over the radial layers), then runs
    ``artes_amd.atmosphere.build`` (atmosphere.py), which writes ``atmosphere.fits``.
    ``wavelengths``: optional index subset of the fixture's wavelengths."""
    from . import atmosphere, gas

    z = np.load(fixture)
    opd = os.path.join(directory, "opacity")
    os.makedirs(opd, exist_ok=True)
    gas.write_pt_file(directory, z["pressure"], z["temperature"])
    sel = slice(None) if wavelengths is None else np.asarray(wavelengths)
    for layer, opacity in zip(z["layers"], z["opacity"]):
        o = np.ascontiguousarray(opacity[:, sel])
        op.write_opacity_fits(os.path.join(opd, "gas_opacity_%02d.fits" % int(layer)), o,
                              gas.rayleigh_matrix_table(0.0, o.shape[1]))
    with open(os.path.join(directory, "atmosphere.in"), "w") as f:
        f.write(SELF_LUMINOUS_IN.format(theta=theta, phi=phi))
    return atmosphere.build(directory)

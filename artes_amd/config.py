"""``artes.in`` / ``-k key=value`` configuration, restating ARTES' keyword system.

Reference: defaults ``ARTES.f90:280-314``; comment rule ``ARTES.f90:384-397``;
``get_key_value`` ``ARTES.f90:4502-4517``; keyword table ``input_parameters``
``ARTES.f90:4361-4500``; ``-k`` overrides applied after the file
(``ARTES.f90:400``, ``4295-4303``).

Semantics kept on purpose:
* keys are applied in file order, so ``star:theta`` only takes effect when
  ``star:direction=on`` was seen earlier (``ARTES.f90:4430-4441``);
* Fortran ``(e50.0)`` reads accept ``1d-5``; a blank value reads as 0;
* angles are converted to radians and ``detector:theta`` / ``star:theta`` are
  clamped to [1e-3, pi-1e-3] exactly as the reference does;
* an unknown key is fatal (the reference prints and calls ``exit(0)``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field, fields

PI = 4.0 * math.atan(1.0)
K_B = 1.3806488e-23
SB = 5.670373e-8
HH = 6.62606957e-34
CC = 2.99792458e8
R_SUN = 6.95500e8
PC = 3.08572e16
AU = 1.49598e11


class ConfigError(ValueError):
    """Raised where the reference would print an error and ``exit(0)``."""


def _fortran_real(value: str) -> float:
    v = value.strip()
    if not v:
        return 0.0
    return float(v.replace("d", "e").replace("D", "E"))


def _fortran_int(value: str) -> int:
    v = value.strip()
    if not v:
        return 0
    return int(v)


@dataclass
class RunConfig:
    """The reference's module-level run parameters (``ARTES.f90:18-56``)."""

    log_file: bool = False
    email: str = ""
    photon_source: int = 1            # 1 = star, 2 = planet
    fstop: float = 1.0e-5
    photon_minimum: float = 1.0e-20
    thermal_weight: bool = True
    photon_scattering: bool = True
    photon_emission: int = 1          # 1 = isotropic, 2 = biased
    photon_bias: float = 0.8
    t_star: float = 5800.0
    r_star: float = R_SUN
    stellar_direction: bool = False
    theta_star: float = PI / 2.0
    phi_star: float = 0.0
    surface_albedo: float = 0.0
    oblateness: float = 0.0
    orbit: float = 5.0 * AU
    ring: bool = False
    phase_curve: bool = False
    spectrum: bool = False
    imaging_mono: bool = False
    imaging_broad: bool = False
    det_theta: float = 90.0           # NB: the reference default is 90 *before* conversion
    det_phi: float = 90.0             #     (``ARTES.f90:307-308``); see ``finalize_detector``
    nx: int = 25
    ny: int = 25
    distance_planet: float = 10.0 * PC
    flow_global: bool = False
    flow_theta: bool = False
    engine: dict = field(default_factory=dict)   # engine:<key>=<int> -- launch tuning (not a reference key)
    applied: list = field(default_factory=list)

    def copy(self) -> "RunConfig":
        c = RunConfig(**{f.name: getattr(self, f.name) for f in fields(self) if f.name not in ("applied", "engine")})
        c.applied = list(self.applied)
        c.engine = dict(self.engine)
        return c

    # ------------------------------------------------------------------ keys
    def apply(self, key: str, value: str) -> None:
        """``input_parameters`` (``ARTES.f90:4361-4500``)."""
        k = key.strip()
        v = value.strip()
        self.applied.append((k, v))
        if k == "general:log":
            if v == "on":
                self.log_file = True
            elif v == "off":
                self.log_file = False
        elif k == "general:email":
            self.email = v
        elif k == "photon:source":
            if v == "star":
                self.photon_source = 1
            elif v == "planet":
                self.photon_source = 2
        elif k == "photon:fstop":
            self.fstop = _fortran_real(v)
        elif k == "photon:minimum":
            self.photon_minimum = _fortran_real(v)
        elif k == "photon:weight":
            if v == "on":
                self.thermal_weight = True
            elif v == "off":
                self.thermal_weight = False
        elif k == "photon:scattering":
            if v == "on":
                self.photon_scattering = True
            elif v == "off":
                self.photon_scattering = False
        elif k == "photon:emission":
            if v == "isotropic":
                self.photon_emission = 1
            elif v == "biased":
                self.photon_emission = 2
        elif k == "photon:bias":
            self.photon_bias = _fortran_real(v)
        elif k == "star:temperature":
            self.t_star = _fortran_real(v)
        elif k == "star:radius":
            self.r_star = _fortran_real(v) * R_SUN
        elif k == "star:direction":
            if v == "on":
                self.stellar_direction = True
            elif v == "off":
                self.stellar_direction = False
        elif k == "star:theta":
            if self.stellar_direction:
                t = _fortran_real(v) * PI / 180.0
                if t < 1.0e-3:
                    t = 1.0e-3
                if t > PI - 1.0e-3:
                    t = PI - 1.0e-3
                self.theta_star = t
        elif k == "star:phi":
            if self.stellar_direction:
                self.phi_star = _fortran_real(v) * PI / 180.0
        elif k == "planet:surface_albedo":
            self.surface_albedo = _fortran_real(v)
        elif k == "planet:oblateness":
            self.oblateness = _fortran_real(v)
        elif k == "planet:orbit":
            self.orbit = _fortran_real(v) * AU
        elif k == "planet:ring":
            if v == "on":
                self.ring = True
            elif v == "off":
                self.ring = False
        elif k == "detector:type":
            if v == "phase":
                self.phase_curve = True
            elif v == "spectrum":
                self.spectrum = True
            elif v == "imaging_mono":
                self.imaging_mono = True
            elif v == "imaging_broad":
                self.imaging_broad = True
        elif k == "detector:theta":
            t = _fortran_real(v) * PI / 180.0
            if t < 1.0e-3:
                t = 1.0e-3
            if t > PI - 1.0e-3:
                t = PI - 1.0e-3
            self.det_theta = t
        elif k == "detector:phi":
            self.det_phi = _fortran_real(v) * PI / 180.0
        elif k == "detector:pixel":
            n = _fortran_int(v)
            self.nx = n
            self.ny = n
        elif k == "detector:distance":
            self.distance_planet = _fortran_real(v) * PC
        elif k == "output:flow_global":
            if v == "on":
                self.flow_global = True
            elif v == "off":
                self.flow_global = False
        elif k == "output:flow_latitudinal":
            if v == "on":
                self.flow_theta = True
            elif v == "off":
                self.flow_theta = False
        elif k.startswith("engine:"):
            # An extension of the reference's keyword table: engine:<tuning key>=<integer> passes an
            # artes_set_tuning key of this engine to every grid the run creates (e.g.
            # -k engine:det_ordered=1 for bit-reproducible detector images; include/artes_amd.h)
            from .engine import TUNING_KEYS

            name = k[len("engine:"):]
            if name not in TUNING_KEYS:
                raise ConfigError(f"Wrong keyword found in input file: {k}")
            try:
                self.engine[name] = int(v)
            except ValueError:
                raise ConfigError(f"Wrong value for {k}: {v}") from None
        else:
            raise ConfigError(f"Wrong keyword found in input file: {k}")

    @property
    def mode(self) -> str:
        """Run-mode dispatch order of ``run`` (``ARTES.f90:132-263``)."""
        if self.spectrum:
            return "spectrum"
        if self.imaging_broad:
            return "imaging_broad"
        if self.phase_curve:
            return "phase"
        if self.imaging_mono:
            return "imaging_mono"
        return "none"


def split_key_value(line: str) -> tuple[str, str]:
    """``get_key_value`` (``ARTES.f90:4502-4517``): split at the first '=', strip quotes."""
    line = line.rstrip("\n").rstrip()
    idx = line.find("=")
    if idx < 0:
        return line.strip(), ""
    key = line[:idx]
    value = line[idx + 1:].rstrip()
    if value[:1] in ("'", '"'):
        value = value[1:-1] if len(value) >= 2 else ""
    return key, value


def is_comment(line: str) -> bool:
    """Comment rule of ``ARTES.f90:390``: first char in ``*-=`` or a blank line."""
    first = line[:1]
    return first in ("*", "-", "=") or len(line.rstrip()) == 0


def read_artes_in(path: str, cfg: RunConfig | None = None) -> RunConfig:
    cfg = cfg if cfg is not None else RunConfig()
    with open(path, "r") as f:
        for line in f:
            line = line.rstrip("\n")
            if is_comment(line):
                continue
            key, value = split_key_value(line)
            cfg.apply(key, value)
    return cfg

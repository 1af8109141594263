"""ctypes mirror of ``include/artes_amd.h`` (struct layouts and constants).

Shared by the product binding (``artes_amd.engine``) and the test-side oracle
binding (``oracle/oracle.py``) so both are driven with byte-identical inputs.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

ARTES_NUM_ERR = 64
ARTES_NUM_COUNTERS = 8
ARTES_NUM_TOTALS = 10      # [0..3] sum T_p, [4..7] sum T_p^2, [8] flux_emitted, [9] flux_exit
ARTES_ABI_VERSION = 6
ARTES_TRACE_FIELDS = 8    # artes_run_trace record: I, scatters, crossings, end state, -Q, U, V, 0
COUNTER_NAMES = ("crossings", "scatters", "peels", "packets", "exited", "absorbed", "dropped", "detected")

_dp = C.POINTER(C.c_double)


class GridDesc(C.Structure):
    _fields_ = [
        ("nr", C.c_int32), ("ntheta", C.c_int32), ("nphi", C.c_int32), ("nwav", C.c_int32),
        ("radial", _dp), ("theta_deg", _dp), ("phi_deg", _dp), ("wavelength_um", _dp),
        ("kappa_sca", _dp), ("kappa_abs", _dp), ("scatter", _dp), ("temperature", _dp),
        ("oblateness", C.c_double),
    ]


class RunParams(C.Structure):
    _fields_ = [
        ("wl_index", C.c_int32), ("nx", C.c_int32), ("ny", C.c_int32), ("photon_source", C.c_int32),
        ("photon_scattering", C.c_int32), ("phase_far", C.c_int32), ("stellar_direction", C.c_int32),
        ("cell_depth", C.c_int32),
        ("det_theta", C.c_double), ("det_phi", C.c_double), ("x_max", C.c_double), ("y_max", C.c_double),
        ("fstop", C.c_double), ("photon_minimum", C.c_double), ("surface_albedo", C.c_double),
        ("theta_star", C.c_double), ("phi_star", C.c_double),
        ("photon_emission", C.c_int32), ("thermal_weight", C.c_int32), ("ring", C.c_int32), ("packet_moments", C.c_int32),
        ("photon_bias", C.c_double),
    ]


def _ptr(a: np.ndarray | None):
    if a is None:
        return C.cast(None, _dp)
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


class GridArrays:
    """Owns C-contiguous float64 copies of the atmosphere arrays and the GridDesc pointing at them."""

    def __init__(self, atm: dict, oblateness: float = 0.0):
        def f64(x):
            return np.ascontiguousarray(np.asarray(x, dtype=np.float64))

        self.radial = f64(atm["radial"])
        self.theta = f64(atm["theta"])
        self.phi = f64(atm["phi"])
        self.wavelength = f64(atm["wavelength"])
        self.kappa_sca = f64(atm["scattering"])
        self.kappa_abs = f64(atm["absorption"])
        sm = np.asarray(atm["scattermatrix"])
        self.scatter = sm if (sm.dtype == np.float64 and sm.flags.c_contiguous) else np.ascontiguousarray(sm, dtype=np.float64)
        t = atm.get("temperature")
        self.temperature = f64(t) if t is not None else None
        self.nr = self.radial.size - 1
        self.ntheta = self.theta.size - 1
        self.nphi = self.phi.size
        self.nwav = self.wavelength.size
        want = (self.nwav, self.nphi, self.ntheta, self.nr)
        if self.kappa_sca.shape != want or self.kappa_abs.shape != want:
            raise ValueError(f"opacity arrays must have shape {want}, got {self.kappa_sca.shape}/{self.kappa_abs.shape}")
        if self.scatter.shape != (180, 16) + want:
            raise ValueError(f"scatter matrix must have shape {(180, 16) + want}, got {self.scatter.shape}")
        self.desc = GridDesc(self.nr, self.ntheta, self.nphi, self.nwav,
                             _ptr(self.radial), _ptr(self.theta), _ptr(self.phi), _ptr(self.wavelength),
                             _ptr(self.kappa_sca), _ptr(self.kappa_abs), _ptr(self.scatter),
                             _ptr(self.temperature), float(oblateness))

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

"""Energy-transport diagnostics (output:flow_global / output:flow_latitudinal,
ARTES.f90:4992-5047, written by write_output 3715-3768).

CPU: the oracle's restatement against exact bookkeeping identities (the flow files of
the reference's frozen runs do not exist -- those runs had the diagnostics off -- so
this row is parity unpinned against the reference itself).  GPU: the engine's
accumulators against the oracle's on packet-identical trajectories.
"""

import numpy as np
import pytest

from artes_amd import driver, fitsio, runner, synthetic


def _cfg(**kv):
    cfg = driver.default_config()
    for k, v in kv.items():
        cfg.apply(k.replace("__", ":"), v)
    return cfg


def _params(atm, cfg):
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    return driver.run_params(cfg, det, 0, cell_depth=-1)


CASES = {
    "ray3d_star": (lambda: synthetic.make("ray", nr=10, ntheta=6, nphi=8, tau=1.0), {}),
    "thermal": (lambda: synthetic.make_thermal(nr=10, ntheta=6, nphi=8, tau_abs=1.0, tau_sca=2.0),
                dict(photon__source="planet")),
    "thermal_surface": (lambda: synthetic.make_thermal(nr=8, ntheta=4, nphi=4, tau_abs=0.5, tau_sca=0.5),
                        dict(photon__source="planet", planet__surface_albedo="0.7")),
}


def test_flow_is_pure_diagnostics(oracle_mod):
    atm = synthetic.make("ray", nr=8, ntheta=4, nphi=4, tau=1.0)
    g = oracle_mod.OracleGrid(atm)
    p = _params(atm, _cfg())
    a = g.run(p, 0, 4000, 7, threads=2)
    b = g.run_flow(p, 0, 4000, 7, threads=2)
    for x, y in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y)
    fg, ft = b[4], b[5]
    assert fg.shape == (4, 4, 8, 3) and ft.shape == (4, 4, 8, 4)
    assert np.abs(fg).sum() > 0 and ft.sum() > 0 and np.all(ft >= 0)


def test_flow_bookkeeping_identities(oracle_mod):
    """Planet source: the Stokes I leaving the top cells upward is flux_exit exactly; with
    a black surface, what crosses the surface downward never comes back up."""
    atm = synthetic.make_thermal(nr=8, ntheta=4, nphi=4, tau_abs=1.0, tau_sca=1.0)
    g = oracle_mod.OracleGrid(atm)
    cfg = _cfg(photon__source="planet")
    p = _params(atm, cfg)
    det, tot, cnt, err, fg, ft = g.run_flow(p, 0, 20000, 11, threads=4)
    assert tot[9] > 0
    assert ft[:, :, -1, 0].sum() == pytest.approx(tot[9], rel=1e-12)
    cd = g.thermal(0, True, False)[0]
    assert ft[:, :, cd, 1].sum() > 0                      # downward through the surface
    assert np.all(ft[:, :, :cd, :] == 0) and np.all(fg[:, :, :cd, :] == 0)
    # downward crossings of the top cells' lower faces are matched by upward crossings
    # of the same faces counted one layer down, plus what was emitted in between
    assert ft[:, :, -2, 0].sum() > 0 and ft[:, :, -1, 1].sum() > 0


def test_flow_output_normalisation():
    rng = np.random.default_rng(3)
    f = rng.normal(size=(2, 3, 5, 3))
    f[0, 0, 4] = 0.0
    out = driver.flow_global_output(f, 2)
    assert np.all(out[:, :, :2] == 0)
    n = np.linalg.norm(out[:, :, 2:], axis=-1)
    assert np.allclose(n[n > 0], 1.0) and np.all(out[0, 0, 4] == 0)
    t = np.abs(rng.normal(size=(2, 3, 5, 4)))
    lat = driver.flow_latitudinal_output(t, 1, 2.0)
    np.testing.assert_array_equal(lat[:, :, 1:], t[:, :, 1:] / 2.0)
    assert np.all(lat[:, :, 0] == 0)


def test_flow_cli_files(tmp_path):
    """output:flow_global / output:flow_latitudinal through the drop-in CLI (oracle as the
    transport): the top cells' upward column of flow_latitudinal.fits sums to 1 (it is
    normalised by the total emergent flux)."""
    from tests.test_cli import OracleTransport, _make_thermal_input

    _make_thermal_input(tmp_path)
    assert runner.run(["hot", "20000", "-o", "fl", "-k", "output:flow_global=on", "-k", "output:flow_latitudinal=on",
                       "--seed", "3"], root=str(tmp_path), transport_factory=OracleTransport) == 0
    out = tmp_path / "output" / "fl" / "output"
    fg = fitsio.read(out / "flow_global.fits")[0].data
    ft = fitsio.read(out / "flow_latitudinal.fits")[0].data
    assert fg.shape == (4, 4, 8, 3) and ft.shape == (4, 4, 8, 4)
    assert ft[:, :, -1, 0].sum() == pytest.approx(1.0, rel=1e-12)
    n = np.linalg.norm(fg, axis=-1)
    assert np.allclose(n[n > 0], 1.0)
    # net transport in the top layer is outward
    assert fg[:, :, -1, 0].mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_flow_matches_oracle_on_gpu(require_gpu, oracle_mod, case):
    from artes_amd.engine import Grid

    make, kv = CASES[case]
    atm = make()
    cfg = _cfg(**kv)
    p = _params(atm, cfg)
    n, seed = 40000, 99
    grid = Grid(atm, device=0)
    rec = grid.trace(p, 0, n, seed)
    res = grid.run(p, 0, n, seed, flow_global=True, flow_latitudinal=True)
    plain = grid.run(p, 0, n, seed)
    grid.close()
    og = oracle_mod.OracleGrid(atm)
    ref = og.run(p, 0, n, seed, records=True)[4]
    det, tot, cnt, err, fg, ft = og.run_flow(p, 0, n, seed)
    # the flow instantiation transports the same packets (it walks the propagation after
    # the forced interaction forwards only, so sums agree to rounding, not bit for bit)
    np.testing.assert_allclose(res.det, plain.det, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(res.counters.astype(float), plain.counters.astype(float), rtol=1e-4)
    # packet-identical trajectories -> accumulators equal up to summation order
    same = (rec[:, 1] == ref[:, 1]) & (rec[:, 2] == ref[:, 2]) & (rec[:, 3] == ref[:, 3])
    assert same.all(), f"{(~same).sum()} trajectories differ"
    np.testing.assert_allclose(res.flow_latitudinal, ft, rtol=1e-9, atol=1e-12 * np.abs(ft).max())
    np.testing.assert_allclose(res.flow_global, fg, rtol=1e-8, atol=1e-11 * np.abs(fg).max())
    if kv.get("photon__source") == "planet":
        assert res.flow_latitudinal[:, :, -1, 0].sum() == pytest.approx(res.totals[9], rel=1e-12)

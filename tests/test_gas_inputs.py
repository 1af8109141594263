"""Input path of the thermal configurations: the restated
pressure-temperature generators, the gas and molecular opacity generators
(artes_amd.gas, restating python/opacityGas.py, opacityMolecules.py,
pressureTemperature*.py) and atmosphere.py's gas branch, end to end into the oracle.

The molecular tests read the reference's own data tables (dat/molecules/PTgrid.dat,
opacity_aver_NNNN.dat, dat/absorption/methane.dat) as inputs when this container has
them; they are skipped elsewhere.  The reference generators themselves (Python 2 +
astropy) cannot run here, so the interpolation is checked against its defining
properties (exact at grid nodes, log-bilinear in between).
"""

import math
import os

import numpy as np
import pytest

from artes_amd import atmosphere, driver, gas

REF_DAT = "/root/reference/dat"
MOL = os.path.join(REF_DAT, "molecules")
need_dat = pytest.mark.skipif(not os.path.isdir(MOL), reason="reference data tables not present")


def test_pt_profiles():
    p, t = gas.pt_isothermal(800.0, 1e-3, 1e2, 40)
    assert p.size == 40 and p[0] == pytest.approx(1e-3) and p[-1] == pytest.approx(1e2) and np.all(t == 800.0)
    p, t = gas.pt_self_luminous(t_eff=800.0, kappa=1e-2, log_g=3.4, p_min=1e-3, p_max=1e2, levels=20)
    tau = 1e-2 * p * 1e6 / 10 ** 3.4
    np.testing.assert_allclose(t, (0.75 * 800.0 ** 4 * (2.0 / 3.0 + tau)) ** 0.25, rtol=1e-14)
    assert np.all(np.diff(t) > 0)          # hotter with depth
    # Eddington: T = Teff where tau = 2/3
    assert (0.75 * 800.0 ** 4 * (4.0 / 3.0)) ** 0.25 == pytest.approx(800.0)


@need_dat
def test_molecule_interpolation_exact_on_grid_nodes():
    grid = gas.read_pt_grid(MOL)
    for row in (5, 200, 700):
        fnum, p, t = grid[row]
        idx = gas.pt_corners(grid, math.log10(p), t)
        # 10**log10(p) != p in the last bit, so the reference's equality test misses and the
        # node's pressure row pair is interpolated with ~1e-16 weight on the neighbour
        assert row in idx and idx[2] == idx[0] and idx[3] == idx[1]
        ops = [gas.read_grid_opacity(MOL, k + 1)[1] for k in idx]
        got = gas.interpolate_pt(grid, p, t, idx, ops)
        want = gas.read_grid_opacity(MOL, int(fnum))[1]
        ok = want > 1e-300
        np.testing.assert_allclose(got[ok], want[ok], rtol=1e-10)


@need_dat
def test_molecule_interpolation_log_bilinear_centre():
    grid = gas.read_pt_grid(MOL)
    # a cell of the P-T grid: two temperatures, two pressures present at both
    t_vals = np.unique(grid[:, 2])
    t1, t2 = t_vals[10], t_vals[11]
    p_vals = np.intersect1d(grid[grid[:, 2] == t1, 1], grid[grid[:, 2] == t2, 1])
    p1, p2 = p_vals[3], p_vals[4]
    pc, tc = math.sqrt(p1 * p2), math.sqrt(t1 * t2)      # centre in log P, log T
    idx = gas.pt_corners(grid, math.log10(pc), tc)
    corners = {(grid[k, 1], grid[k, 2]) for k in idx}
    assert corners == {(p1, t1), (p1, t2), (p2, t1), (p2, t2)}
    ops = [gas.read_grid_opacity(MOL, k + 1)[1] for k in idx]
    got = gas.interpolate_pt(grid, pc, tc, idx, ops)
    logs = np.log10(np.maximum(np.array(ops), 1e-500))
    logs[logs < -500] = -500
    np.testing.assert_allclose(np.log10(got), logs.mean(axis=0), rtol=0, atol=1e-9)


@need_dat
def test_gas_opacity_methane():
    op, sc = gas.gas_opacity(os.path.join(REF_DAT, "absorption", "methane.dat"), wavelength_min=0.5,
                             wavelength_max=0.6, manual_step=0.01)
    assert op.shape[0] == 4 and 5 <= op.shape[1] <= 12
    np.testing.assert_allclose(op[1], op[2] + op[3], rtol=1e-14)
    # Rayleigh scattering scales as lambda^-4 up to the H2 dispersion term
    ratio = op[3, 0] / op[3, -1] * (op[0, 0] / op[0, -1]) ** 4
    assert 1.0 < ratio < 1.02
    # normalised matrix: 2 pi int P11 sin = 1
    ang = (np.arange(180) + 0.5) * math.pi / 180
    assert 2 * math.pi * np.sum(sc[:, 0, 0] * np.sin(ang)) * math.pi / 180 == pytest.approx(1.0, rel=2e-3)


@need_dat
def test_self_luminous_atmosphere_end_to_end(tmp_path, oracle_mod):
    """pressureTemperature + molecular opacities + atmosphere.py gas branch -> atmosphere.fits,
    then the planet source on the oracle: emitted luminosity = sum of cell luminosities."""
    d = tmp_path / "input" / "self_luminous"
    d.mkdir(parents=True)
    p, t = gas.pt_self_luminous(t_eff=800.0, levels=12)
    gas.write_pt_file(str(d), p, t)
    paths = gas.write_molecule_opacities(str(d), p, t, MOL, wavelength_min=1.6, wavelength_max=1.62)
    assert len(paths) == 12
    (d / "atmosphere.in").write_text(
        "[grid]\nradius: 1.\nradial:\ntheta:\nphi:\n\n[composition]\ngas: on\nmolweight: 2.02\nlog_g: 3.4\n"
        "ring:\n")
    atm = atmosphere.build(str(d))
    assert (d / "atmosphere.fits").exists()
    assert atm["absorption"].shape[1:] == (1, 1, 11)
    np.testing.assert_allclose(atm["temperature"][0, 0], np.asarray(t)[::-1][:11], rtol=1e-12)
    assert np.all(atm["absorption"] > 0) and np.all(atm["scattering"] > 0)
    g = oracle_mod.OracleGrid(atm)
    cfg = driver.default_config()
    cfg.apply("photon:source", "planet")
    cfg.apply("detector:pixel", "5")
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    prm = driver.run_params(cfg, det, 0, cell_depth=-1)
    n = 50000
    d_, tot, cnt, err, _ = g.run(prm, 0, n, 3)
    cd, total, lum = g.thermal(0, True, False)
    assert tot[8] * total / n == pytest.approx(lum.sum(), rel=0.03)
    assert d_[0, 0].sum() > 0

"""The gas + Mie-cloud input of tests/test_gpu_cloudy.py (BASELINE configs[3]'s shape),
checked on the CPU: built through atmosphere.build from the restated generators, the
cloud mixed into the gas by extinction weight (atmosphere.py:366-369), and transported
by the oracle without errors at every wavelength."""

import numpy as np

from artes_amd import atmosphere, driver, synthetic


def test_cloudy_atmosphere(tmp_path, oracle_mod):
    d = tmp_path / "input" / "cloudy"
    atm = synthetic.make_cloudy(str(d))
    back = atmosphere.read_atmosphere_fits(str(d / "atmosphere.fits"))
    for k in atmosphere.HDU_ORDER:
        np.testing.assert_array_equal(back[k], atm[k])
    nwav, nphi, nth, nr = atm["scattering"].shape
    assert (nwav, nphi, nth, nr) == (3, 6, 6, 16)
    ext = atm["scattering"] + atm["absorption"]
    h = np.diff(atm["radial"])
    clear = (ext[:, 5, 0, :] * h).sum(-1)
    cloudy = (ext[:, 1, 2, :] * h).sum(-1)
    assert np.all(np.diff(clear) < 0)                     # Rayleigh: thinner to the red
    assert np.all(cloudy > clear + 1.0)                   # the cloud adds optical depth
    m = atm["scattermatrix"].reshape(180 * 16, -1)
    distinct = {m[:, k].tobytes() for k in range(m.shape[1])}
    assert len(distinct) == 1 + 8 * 3                     # the clear-gas Rayleigh matrix + 8 cloudy layers x 3
    # outside the cloud the gas matrix; inside, the extinction-weighted mixture
    np.testing.assert_array_equal(atm["scattermatrix"][:, :, 0, 5, 0, 0], atm["scattermatrix"][:, :, 0, 4, 5, 15])
    og = oracle_mod.OracleGrid(atm)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    for wl in range(nwav):
        p = driver.run_params(cfg, det, wl, cell_depth=og.cell_depth(wl))
        dd, tot, cnt, err, _ = og.run(p, 0, 5000, 9 + wl)
        assert not np.any(err) and dd[0, 0].sum() > 0

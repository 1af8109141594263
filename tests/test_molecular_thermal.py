"""BASELINE configs[4] on the HIP path: self-luminous thermal emission through P-T
dependent molecular opacities (opacityMolecules.py), 100 wavelengths.

The input is built through the restated setup path from the committed opacity fixture
tests/golden/molecular/self_luminous_100wl.npz (tools/make_molecular_fixture.py, made
in the build container from the reference's dat/molecules with
artes_amd.gas.molecule_opacities, the restatement of opacityMolecules.py:120-300; the
fixture is pinned to that generator by test_fixture_matches_generator wherever the data
tables are present).  The thermal source is parity-unpinned against the reference itself
(its frozen runs are star-source only): the GPU engine is compared with the CPU oracle,
packet by packet (same xoroshiro128++ streams) and through the `spectrum` CLI.
"""

import os

import numpy as np
import pytest

from artes_amd import driver, runner, stats, synthetic
from conftest import GOLDEN

FIXTURE = os.path.join(GOLDEN, "molecular", "self_luminous_100wl.npz")
MOL = "/root/reference/dat/molecules"

ARTES_IN = """photon:source=planet
photon:fstop=1d-5
photon:minimum=1d-20
detector:type=spectrum
detector:theta=90
detector:phi=90
detector:distance=10
"""


@pytest.fixture(scope="module")
def self_luminous(tmp_path_factory):
    root = tmp_path_factory.mktemp("sl")
    d = root / "input" / "sl"
    atm = synthetic.make_self_luminous(str(d), FIXTURE)
    (d / "artes.in").write_text(ARTES_IN)
    return root, d, atm


def test_fixture_shape_and_profile():
    z = np.load(FIXTURE)
    assert z["opacity"].shape == (20, 4, 100)
    np.testing.assert_allclose(z["opacity"][:, 1], z["opacity"][:, 2] + z["opacity"][:, 3], rtol=1e-14)
    assert np.all(np.diff(z["opacity"][0, 0]) > 0)                     # wavelengths ascending
    assert z["opacity"][0, 0, 0] >= 1.0 and np.all(z["temperature"] > 600)


@pytest.mark.skipif(not os.path.isdir(MOL), reason="reference data tables not present")
def test_fixture_matches_generator():
    import sys

    from conftest import ROOT

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_molecular_fixture as mk

    d = mk.build(MOL)
    z = np.load(FIXTURE)
    for k in ("pressure", "temperature", "layers", "opacity"):
        np.testing.assert_array_equal(d[k], z[k], err_msg=k)


def test_atmosphere_from_fixture(self_luminous):
    _, d, atm = self_luminous
    assert (d / "atmosphere.fits").exists()
    assert atm["scattering"].shape == (100, 4, 6, 19)
    assert np.all(atm["absorption"] > 0) and np.all(atm["scattering"] > 0)
    # the gas branch orders the layers bottom-up: hottest (deepest) first
    assert np.all(np.diff(atm["temperature"][0, 0]) < 0)


def test_oracle_spectrum_cli_plumbing(self_luminous):
    """The 100-wavelength `spectrum` run on the CPU oracle through the drop-in CLI: one
    spectrum line and one luminosity line per wavelength, emergent < emitted."""
    from test_cli import OracleTransport

    root, _, _ = self_luminous
    assert runner.run(["sl", "300", "-o", "o_cpu", "--seed", "3"], root=str(root),
                      transport_factory=OracleTransport) == 0
    out = root / "output" / "o_cpu" / "output"
    spec = [l for l in (out / "spectrum.dat").read_text().splitlines() if l.strip() and "#" not in l]
    lum = [l for l in (out / "luminosity.dat").read_text().splitlines() if l.strip() and "#" not in l]
    assert len(spec) == 100 and len(lum) == 100
    rows = np.array([[float(x) for x in l.split()] for l in lum])
    assert np.all(rows[:, 1] > 0) and np.all(rows[:, 2] < rows[:, 1])


@pytest.mark.gpu
@pytest.mark.parametrize("wl", [0, 37, 99])
def test_molecular_thermal_trajectories_match_oracle(require_gpu, oracle_mod, self_luminous, wl):
    from artes_amd.engine import Grid

    _, _, atm = self_luminous
    cfg = driver.default_config()
    cfg.apply("photon:source", "planet")
    cfg.apply("detector:type", "spectrum")
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    p = driver.run_params(cfg, det, wl, cell_depth=-1)
    n = 20000
    grid = Grid(atm, device=0)
    og = oracle_mod.OracleGrid(atm)
    assert grid.thermal(wl)[0] == og.thermal(wl)[0]                      # thermal cell_depth
    gpu = grid.trace(p, 0, n, 100 + wl)
    ref = og.run(p, 0, n, 100 + wl, records=True)[4]
    grid.close()
    same = stats.records_agree(gpu, ref)
    short = ref[:, 1] <= 20
    assert same[short].mean() >= 0.999 and same.mean() >= 0.99, (wl, same.mean(), same[short].mean())
    assert gpu[:, 0].sum() > 0


@pytest.mark.gpu
def test_molecular_spectrum_cli_gpu_matches_oracle(require_gpu, self_luminous):
    """All 100 wavelengths through the drop-in CLI on the GPU and on the oracle, same seeds:
    spectrum.dat and luminosity.dat are sums over the same packets."""
    from test_cli import OracleTransport

    root, _, _ = self_luminous
    n = "2000"
    assert runner.run(["sl", n, "-o", "g", "--seed", "5"], root=str(root)) == 0
    assert runner.run(["sl", n, "-o", "o", "--seed", "5"], root=str(root), transport_factory=OracleTransport) == 0

    def rows(run, f):
        txt = (root / "output" / run / "output" / f).read_text().splitlines()
        return np.array([[float(x) for x in l.split()] for l in txt if l.strip() and "#" not in l])

    for f in ("spectrum.dat", "luminosity.dat"):
        g, o = rows("g", f), rows("o", f)
        assert g.shape == o.shape and g.shape[0] == 100, f
        np.testing.assert_allclose(g[:, 0], o[:, 0], rtol=1e-12)
        scale = np.abs(o[:, 1:]).max(axis=0)
        assert np.all(np.abs(g[:, 1:] - o[:, 1:]) <= 1e-3 * scale + 1e-3 * np.abs(o[:, 1:])), f
    assert (root / "output" / "g" / "error.log").read_text() == (root / "output" / "o" / "error.log").read_text()

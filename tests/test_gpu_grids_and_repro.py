"""Grids whose face tables exceed k_trace's LDS budget, and bit-reproducible detector images.

* Face tables beyond 64 KiB: k_trace stages its face records in LDS up to
  64 KiB and reads them from a global (L2-resident) copy beyond that (the GTAB kernels,
  kernel_trace.hpp).  The reference allocates any grid (ARTES.f90:2237-2307, 58-91): a fine
  P-T profile of ~2000 radial faces must run and match the oracle packet by packet.
* det_ordered: the detector planes 0-11 (Stokes sums, squares, counts)
  accumulated as 128-bit fixed-point integers (kernel_event.hpp, fix_add), so two identical runs
  give identical bits -- through the C ABI and through the drop-in CLI
  (-k engine:det_ordered=1 -> identical stokes.fits, error.fits, photometry.dat).
"""

import hashlib
import os

import numpy as np
import pytest

from artes_amd import atmosphere, driver, runner, stats, synthetic

pytestmark = pytest.mark.gpu


def _grid_and_params(atm):
    from artes_amd.engine import Grid

    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    grid = Grid(atm, device=0)
    p = driver.run_params(cfg, det, 0, cell_depth=grid.cell_depth(0))
    return grid, p


@pytest.mark.parametrize("name,spec,n", [("ray3d", dict(nr=2100, ntheta=4, nphi=4), 4000),
                                         ("hg", dict(nr=4000), 3000)])
def test_face_tables_beyond_lds_match_oracle(require_gpu, oracle_mod, name, spec, n):
    """2100 radial faces x 4 x 4 (101 KiB of face tables) and a 4000-shell radial-only grid
    (192 KiB): the run is not refused, takes the global-table kernel and its trajectories match
    the oracle's."""
    from artes_amd.engine import Grid

    atm = synthetic.make_config(name, share_matrix=True, **spec)
    grid, p = _grid_and_params(atm)
    gpu = grid.trace(p, 0, n, 2024)
    assert grid.last_launch().split()[0].endswith(",1>"), grid.last_launch()   # k_trace<...,1>: GTAB
    ref = oracle_mod.OracleGrid(atm).run(p, 0, n, 2024, records=True)[4]
    same = stats.records_agree(gpu, ref)
    short = ref[:, 1] <= 20
    assert same[short].mean() >= 0.999 and same.mean() >= 0.99, (same.mean(), same[short].mean())
    assert gpu[:, 2].mean() > 2 * spec["nr"]   # (every packet crosses the fine shells)
    res = grid.run(p, 0, 200000, 7)
    assert res.err[:57].sum() == 0 and res.det[0, 0].sum() > 0
    grid.close()


def test_global_face_tables_equal_lds_tables(require_gpu):
    """trace_gtab = 1 forces the global-table kernel on a grid whose tables fit in LDS: the same
    arithmetic on the same values, so the same packet records and counters."""
    atm = synthetic.make_config("ray3d", nr=10, ntheta=6, nphi=8)
    grid, p = _grid_and_params(atm)
    lds = grid.trace(p, 0, 20000, 99)
    r_lds = grid.run(p, 0, 300000, 5)
    assert not grid.last_launch().split()[0].endswith(",1>")
    grid.set_tuning(trace_gtab=1)
    glob = grid.trace(p, 0, 20000, 99)
    r_glob = grid.run(p, 0, 300000, 5)
    assert grid.last_launch().split()[0].endswith(",1>")
    np.testing.assert_array_equal(lds, glob)
    np.testing.assert_array_equal(r_lds.counters, r_glob.counters)
    np.testing.assert_allclose(r_lds.det, r_glob.det, rtol=1e-9, atol=1e-300)


@pytest.mark.parametrize("name,spec,mode", [("ray3d", {}, "image"), ("hg", {}, "image"), ("ray3d", dict(nr=8, ntheta=6, nphi=6), "pixel"),
                                            ("ray3d", dict(nr=8, ntheta=6, nphi=6), "big")])
def test_det_ordered_runs_are_bit_identical(require_gpu, name, spec, mode):
    """Two identical det_ordered calls give the same bits; the image agrees with the
    floating-point accumulation to rounding (the fixed point resolves 2^-80)."""
    atm = synthetic.make_config(name, share_matrix=True, **spec)
    grid, p = _grid_and_params(atm)
    # (the packet-level moments -- diagnostics, off in the CLI and the bench -- stay floating-point
    # sums: planes 12-15 and totals 4-7 are not covered by det_ordered)
    p.packet_moments = 0
    if mode == "pixel":   # a one-pixel detector (spectrum / phase): every peel on one address
        p.nx = p.ny = 1
    if mode == "big":     # 48 x 48 pixels: the fixed-point planes exceed LDS, added to HBM at once (ORD = 1)
        p.nx = p.ny = 48
    base = grid.run(p, 0, 2_000_000, 11)
    grid.set_tuning(det_ordered=1)
    a = grid.run(p, 0, 2_000_000, 11)
    ev = grid.last_launch().split()[1]
    assert ev.endswith(",2>") or ev.endswith(",1>"), ev   # k_event<...,ORD>: fixed point in LDS (2) or HBM (1)
    b = grid.run(p, 0, 2_000_000, 11)
    assert a.det.tobytes() == b.det.tobytes()
    assert a.totals.tobytes() == b.totals.tobytes()
    np.testing.assert_array_equal(a.counters, base.counters)
    np.testing.assert_allclose(a.det, base.det, rtol=1e-10, atol=1e-20)
    grid.close()


ARTES_IN = """photon:source=star
photon:fstop=1d-5
star:temperature=5800
star:radius=1
planet:orbit=5
detector:type=imaging_mono
detector:theta=90
detector:phi=90
detector:pixel=25
detector:distance=10
"""


def test_cli_det_ordered_gives_identical_files(tmp_path, require_gpu):
    """The drop-in CLI with -k engine:det_ordered=1, twice: byte-identical stokes.fits,
    error.fits and photometry.dat."""
    d = tmp_path / "input" / "atm"
    d.mkdir(parents=True)
    (d / "artes.in").write_text(ARTES_IN)
    atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"), synthetic.make_config("ray3d", nr=12, ntheta=8, nphi=8))
    digests = []
    for run in ("a", "b"):
        assert runner.run(["atm", "3e6", "-o", run, "-k", "engine:det_ordered=1", "--seed", "17"], root=str(tmp_path)) == 0
        out = tmp_path / "output" / run / "output"
        digests.append([hashlib.sha256(open(out / f, "rb").read()).hexdigest()
                        for f in ("stokes.fits", "error.fits", "photometry.dat")])
        assert os.path.getsize(tmp_path / "output" / run / "error.log") == 0
    assert digests[0] == digests[1]

"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and the frozen
reference runs.

* Trajectory level: the engine and the oracle draw the same xoroshiro128++ stream per
  packet, so each packet's history (scatterings, cell crossings, end state, peeled
  intensity) must agree; FMA contraction and libm-vs-ocml last-ulp differences may flip
  a rare near-tie decision, so >= 99.9 % of packets must match to 1e-9.  Very long
  histories are chaotic in the last bit (the oracle built with -mfma agrees with itself
  on only 99.87 % of tau=40 packets, mean 62 scatterings), so the criterion applies to
  packets with <= 20 scatterings, and all packets must agree to >= 99 %.
* Statistical level: per-pixel Stokes z-scores against the reference's own images
  (tolerance: Monte-Carlo sigma, honest packet-level variance; see tests/golden/README.md).
"""

import math
import os

import numpy as np
import pytest

from artes_amd import driver, stats, synthetic
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
REF = os.path.join(GOLDEN, "reference_runs")


def _params(cfg, atm, grid_like, **over):
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    p = driver.run_params(cfg, det, 0, cell_depth=grid_like.cell_depth(0))
    for k, v in over.items():
        setattr(p, k, v)
    return det, p


def _agreement(require_gpu, oracle_mod, atm, cfg, n=20000, seed=31337, oblateness=0.0, **over):
    from artes_amd.engine import Grid

    grid = Grid(atm, device=0, oblateness=oblateness)
    og = oracle_mod.OracleGrid(atm, oblateness=oblateness)
    det, p = _params(cfg, atm, og, **over)
    gpu = grid.trace(p, 0, n, seed)
    ref = og.run(p, 0, n, seed, records=True)[4]
    same = stats.records_agree(gpu, ref)
    grid.close()
    return same.mean(), gpu, ref


CASES = {
    "iso_1d": (dict(name="iso"), {}),
    "hg_1d": (dict(name="hg"), {}),
    "ray_3d_small": (dict(name="ray3d", nr=8, ntheta=8, nphi=8), {}),
    "ray_3d_full": (dict(name="ray3d"), {}),
    "ray_theta3_no_plane": (dict(name="ray3d", nr=6, ntheta=3, nphi=5), {}),
    "ray_phi2_wrap": (dict(name="ray3d", nr=6, ntheta=4, nphi=2), {}),
    "hg_thick_surface": (dict(name="hg", tau=40.0), {}),
    "ray_absorbing": (dict(name="ray3d", nr=8, ntheta=4, nphi=4, omega=0.6), {}),
    # fine angular grids: many theta / phi faces within a radial shell, so new traces
    # often step on one family while the others are still set-up bounds (lazy set-up,
    # kernel_trace.hpp); the thick one scatters ~8 times per packet (many new traces)
    "ray_fine_angles": (dict(name="ray3d", nr=24, ntheta=30, nphi=48), {}),
    "ray_fine_thick": (dict(name="ray3d", nr=12, ntheta=18, nphi=24, tau=6.0), {}),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_trajectories_match_oracle(require_gpu, oracle_mod, case):
    spec, over = CASES[case]
    spec = dict(spec)
    name = spec.pop("name")
    atm = synthetic.make_config(name, **spec)
    frac, gpu, ref = _agreement(require_gpu, oracle_mod, atm, driver.default_config(), **over)
    short = ref[:, 1] <= 20
    same = stats.records_agree(gpu, ref)
    assert same[short].mean() >= 0.999 and frac >= 0.99, (case, frac, same[short].mean())
    assert gpu[:, 1].sum() > 0 and gpu[:, 2].sum() > 0


def test_trajectories_other_detector_directions(require_gpu, oracle_mod):
    atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
    cfg = driver.default_config()
    cfg.apply("detector:theta", "30")
    cfg.apply("detector:phi", "200")
    frac, _, _ = _agreement(require_gpu, oracle_mod, atm, cfg)
    assert frac >= 0.999


def test_trajectories_stellar_direction_and_phase_far(require_gpu, oracle_mod):
    atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
    cfg = driver.default_config()
    cfg.apply("star:direction", "on")
    cfg.apply("star:theta", "60")
    cfg.apply("star:phi", "30")
    frac, _, _ = _agreement(require_gpu, oracle_mod, atm, cfg)
    assert frac >= 0.999
    cfg2 = driver.default_config()
    frac2, _, _ = _agreement(require_gpu, oracle_mod, atm, cfg2, phase_far=1, det_phi=175 * math.pi / 180)
    assert frac2 >= 0.999


def test_trajectories_oblate_planet_and_no_scattering(require_gpu, oracle_mod):
    atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
    frac, _, _ = _agreement(require_gpu, oracle_mod, atm, driver.default_config(), oblateness=0.1)
    assert frac >= 0.999
    frac2, gpu, _ = _agreement(require_gpu, oracle_mod, atm, driver.default_config(), photon_scattering=0)
    assert frac2 == 1.0 and gpu[:, 0].sum() == 0.0


def _run(require_gpu, atm, n, seed, cfg=None, first=0):
    from artes_amd.engine import Grid

    cfg = cfg or driver.default_config()
    grid = Grid(atm, device=0)
    det, p = _params(cfg, atm, grid)
    res = grid.run(p, first, n, seed)
    return grid, det, p, res


def test_counters_and_no_errors(require_gpu):
    atm = synthetic.make_config("ray3d")
    n = 2 * 10**6
    grid, det, p, res = _run(require_gpu, atm, n, 5)
    c = dict(zip(("crossings", "scatters", "peels", "packets", "exited", "absorbed", "dropped", "detected"),
                 res.counters.tolist()))
    assert c["packets"] == n and c["exited"] + c["absorbed"] + c["dropped"] == n and c["dropped"] == 0
    assert c["crossings"] / n == pytest.approx(109.6, rel=0.01) and c["scatters"] / n == pytest.approx(2.56, abs=0.02)
    assert res.err.sum() == 0
    assert np.all(res.det[2, 0] == res.det[2, 1]) and np.all(res.det[2, 0] == res.det[2, 3])
    assert res.det[2, 0].sum() == c["detected"]


def test_shard_invariance(require_gpu):
    from artes_amd.engine import Grid

    atm = synthetic.make_config("hg")
    grid = Grid(atm, device=0)
    cfg = driver.default_config()
    det, p = _params(cfg, atm, grid)
    a = grid.run(p, 0, 10**6, 77)
    b = grid.run(p, 0, 377777, 77)
    b += grid.run(p, 377777, 10**6 - 377777, 77)
    np.testing.assert_allclose(a.det, b.det, rtol=1e-9, atol=1e-300)
    np.testing.assert_array_equal(a.counters, b.counters)


def test_records_do_not_depend_on_the_split(require_gpu):
    """The engine splits a call's packet ids over 8 XCD-local sub-engines (block b works on
    sub-engine b mod 8); a packet's record must not depend on which sub-engine, slot or
    call carries it: calls of 1, 5 (fewer packets than sub-engines), 13 and 4077 packets
    reproduce the slices of one 4096-packet call bit for bit."""
    from artes_amd.engine import Grid

    atm = synthetic.make_config("ray3d", nr=8, ntheta=8, nphi=8)
    grid = Grid(atm, device=0)
    det, p = _params(driver.default_config(), atm, grid)
    whole = grid.trace(p, 0, 4096, 99)
    parts, first = [], 0
    for n in (1, 5, 13, 4077):
        parts.append(grid.trace(p, first, n, 99))
        first += n
    grid.close()
    np.testing.assert_array_equal(np.concatenate(parts), whole)
    assert (whole[:, 1] > 0).any() and (whole[:, 3] == 1).any()


def test_device_variant_matches_host_variant(require_gpu):
    import torch

    from artes_amd.engine import Grid

    atm = synthetic.make_config("iso")
    grid = Grid(atm, device=0)
    det, p = _params(driver.default_config(), atm, grid)
    host = grid.run(p, 0, 500000, 9)
    d = torch.zeros((4, 4, p.ny, p.nx), dtype=torch.float64, device="cuda:0")
    t2 = torch.zeros(6, dtype=torch.float64, device="cuda:0")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda:0")
    grid.run_device(p, 0, 500000, 9, d.data_ptr(), t2.data_ptr(), cnt.data_ptr(), 0,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_allclose(d.cpu().numpy(), host.det, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(t2.cpu().numpy()[:4], host.totals[4:8], rtol=1e-9)
    assert cnt.cpu().numpy().tolist() == host.counters.astype(np.int64).tolist()


@pytest.mark.parametrize("name,run", [("iso", "t_iso_ARTES_det_1e6"), ("hg", "t_hg_ARTES_det_1e6"),
                                      ("ray3d", "t_ray3d_ARTES_det_1e6")])
def test_statistics_match_reference_runs(require_gpu, name, run):
    """1e8 GPU packets vs the reference's own 1e6-packet images (same inputs)."""
    atm = synthetic.make_config(name, normalizer="simpson", share_matrix=True)
    n = 10**8
    grid, det, p, res = _run(require_gpu, atm, n, 2468)
    E = driver.package_energy(driver.default_config(), 0.7e-6, float(atm["radial"][-1]), n, det.det_phi)
    ref = stats.load_reference_run(os.path.join(REF, run))
    for k in (0, 1, 2):
        cmp = stats.compare_to_reference(res.det, n, E, det.pixel_scale, ref, 10**6, stokes=k)
        if k == 0:
            # Stokes I, SURVEY.md §8(d) / BASELINE.md: RMS(z) <= 1.2 and |mean z| <= 0.1
            assert 0.8 < cmp["rms_z"] <= 1.2 and abs(cmp["mean_z"]) <= 0.1, (k, cmp)
            assert 0.5 < cmp["median_abs_z"] < 0.9 and cmp["frac_gt4"] <= 0.02, (k, cmp)
        elif name != "iso":
            # Q, U, SURVEY.md §8(d): |dX| <= 4 sqrt(s_b^2 + s_r^2) (+ 1e-6 sum I) per pixel.  The
            # mean z of U against ONE 1e6-packet reference image carries that image's own noise
            # (the CPU oracle at 4e6 packets, two seeds: -0.17 / -0.14 against this run, +0.02,
            # +0.06, -0.11 / +0.04, +0.07, -0.07 against the three other reference seeds), so
            # the mean is held to 0.2 here and the per-pixel 4 sigma rule carries the bar
            assert cmp["rms_z"] <= 1.2 and abs(cmp["mean_z"]) <= 0.2, (k, cmp)
            assert cmp["frac_gt4"] == 0.0, (k, cmp)
    ph = driver.photometry(driver.scale_detector(res.det[:3], E)) * 1e-6
    rph = ref["photometry"]
    s_ref = stats.total_sigma_scaled(res.totals, n, E, 10**6) * 1e-6
    for k, col in ((0, 1), (1, 3), (2, 5)):
        assert abs(ph[2 * k] - rph[col]) <= 4 * s_ref[k] + 1e-12 * rph[1], (k, ph[2 * k], rph[col], s_ref[k])
    assert ph[6] == 0.0


def test_gpu_vs_oracle_statistics_1d(require_gpu, oracle_mod):
    """Independent seeds, engine vs oracle: photometry consistent within 4 sigma."""
    atm = synthetic.make_config("hg")
    n_gpu, n_cpu = 2 * 10**7, 2 * 10**6
    grid, det, p, res = _run(require_gpu, atm, n_gpu, 1)
    og = oracle_mod.OracleGrid(atm)
    d2, t2, _, _, _ = og.run(p, 0, n_cpu, 2, threads=16)
    m1 = res.det[0, :3].sum(axis=(1, 2)) / n_gpu
    m2 = d2[0, :3].sum(axis=(1, 2)) / n_cpu
    s1 = stats.total_sigma_raw(res.totals, n_gpu)[:3] / n_gpu
    s2 = stats.total_sigma_raw(t2, n_cpu)[:3] / n_cpu
    assert np.all(np.abs(m1 - m2) <= 4 * np.hypot(s1, s2)), (m1, m2, s1, s2)


@pytest.mark.parametrize("pixels", [5, 101])
def test_detector_image_matches_oracle(require_gpu, oracle_mod, pixels):
    """The detector image of a call against the oracle's, pixel by pixel, at a small detector
    (64 privatised HBM copies: det_copies, transport.hip) and at 101 x 101 pixels, whose copies
    exceed 64 MiB at 64 (32 then); the planes are the reference's detector(:,:,:,1..4)
    accumulation (ARTES.f90:4947-4972), summed in another order, so to rounding."""
    from artes_amd.engine import Grid

    atm = synthetic.make_config("hg")
    cfg = driver.default_config()
    cfg.apply("detector:pixel", str(pixels))
    grid = Grid(atm, device=0)
    og = oracle_mod.OracleGrid(atm)
    det, p = _params(cfg, atm, og)
    assert (p.nx, p.ny) == (pixels, pixels)
    n, seed = 20000, 4711
    res = grid.run(p, 0, n, seed)
    grid.close()
    ref = og.run(p, 0, n, seed)[0]
    assert ref[0, 0].sum() > 0
    for m in range(4):
        scale = np.abs(ref[m]).max()
        np.testing.assert_allclose(res.det[m], ref[m], rtol=1e-9, atol=1e-12 * scale)

"""GPU engine plumbing: both engines (event, persistent) against each other and the
oracle, per-launch timing hooks, launch-knob invariance, C-ABI argument checks."""

import os

import numpy as np
import pytest

from artes_amd import driver, stats, synthetic

pytestmark = pytest.mark.gpu


def _setup(name="ray3d", **spec):
    from artes_amd.engine import Grid

    atm = synthetic.make_config(name, **spec)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    grid = Grid(atm, device=0)
    p = driver.run_params(cfg, det, 0, cell_depth=grid.cell_depth(0))
    return atm, grid, p


def test_event_and_persistent_engines_agree(require_gpu):
    atm, grid, p = _setup(nr=8, ntheta=8, nphi=8)
    ev = grid.trace(p, 0, 20000, 4242)
    assert grid.last_launch().startswith("k_trace<1,0,4,0,4>")   # (512 cells: a coarse grid, 4 steps)
    grid.set_tuning(engine="persistent")
    pe = grid.trace(p, 0, 20000, 4242)
    assert grid.last_launch() == "persistent"
    same = stats.records_agree(ev, pe)
    assert same.mean() >= 0.999


@pytest.mark.parametrize("knobs", [dict(pool=5000), dict(refill=1, static=0), dict(refill=64, static=64),
                                   dict(event_lds=0, det_lds=0), dict(wpe=3), dict(emit_first=0),
                                   dict(emit_first=1, pool=3000), dict(batch=4, batch_min=24),
                                   dict(batch=64, batch_min=1), dict(event_block=256)])
def test_launch_knobs_do_not_change_results(require_gpu, knobs):
    """Pool size, refill policy, trace-list split, LDS staging, occupancy, the k_event block
    shape and the batching of the forced first interaction only change the schedule: per-packet histories and
    all counters are identical."""
    atm, grid, p = _setup("hg")
    base = grid.run(p, 0, 300000, 99)
    grid.close()
    atm, grid, p = _setup("hg")
    grid.set_tuning(**knobs)
    assert grid.tuning() == knobs
    other = grid.run(p, 0, 300000, 99)
    np.testing.assert_array_equal(base.counters, other.counters)
    np.testing.assert_allclose(base.det, other.det, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(base.totals, other.totals, rtol=1e-9)


def test_pool_key_shrinks_an_existing_pool_and_last_launch_names_the_engine(require_gpu, capfd):
    """The "pool" key takes effect on a grid that already holds a larger pool (it is
    reallocated), and artes_last_launch reports "none" for a call that launched nothing
    (ADVICE r05)."""
    atm, grid, p = _setup("hg")
    grid.set_tuning(verbose=1)
    base = grid.run(p, 0, 300000, 99)
    grid.set_tuning(pool=5000)
    other = grid.run(p, 0, 300000, 99)
    err = capfd.readouterr().err
    pools = [int(l.split("pool ")[1].split(",")[0]) for l in err.splitlines() if "event engine: pool" in l]
    assert len(pools) == 2 and pools[0] > 5000 >= pools[1] - 1023, err
    np.testing.assert_array_equal(base.counters, other.counters)
    np.testing.assert_allclose(base.det, other.det, rtol=1e-9, atol=1e-300)
    assert grid.last_launch().startswith("k_trace<0,0,4,0,10>")
    grid.run(p, 0, 0, 99)
    assert grid.last_launch() == "none"


@pytest.mark.parametrize("name,spec", [("hg", {}), ("ray3d", dict(nr=10, ntheta=6, nphi=8, tau=3.0))])
def test_backward_propagation_matches_forward(require_gpu, name, spec):
    """The propagation after the forced first interaction may walk the chord back from
    its far end (kernel_trace.hpp): same interaction point up to rounding, and the
    per-packet crossing counts are reported as the forward walk's."""
    atm, grid, p = _setup(name, **spec)
    back = grid.trace(p, 0, 20000, 31)
    c_back = grid.run(p, 0, 200000, 8).counter("crossings")
    grid.set_tuning(backward=0)
    fwd = grid.trace(p, 0, 20000, 31)
    same = stats.records_agree(back, fwd)
    assert same.mean() >= 0.999
    c_fwd = grid.run(p, 0, 200000, 8).counter("crossings")
    assert c_back == pytest.approx(c_fwd, rel=1e-3)


@pytest.mark.parametrize("name,spec", [("hg", {}), ("ray3d", dict(nr=10, ntheta=6, nphi=8, tau=3.0))])
def test_crossing_counter_is_sum_of_packet_crossings(require_gpu, name, spec):
    """k_trace adds a packet's crossings to the run's counter once per chain of traces
    (kernel_trace.hpp, the chain-end write-back), backward walks counted as the forward
    one: the counter of a run is the sum of the per-packet crossings its records report."""
    atm, grid, p = _setup(name, **spec)
    rec = grid.trace(p, 0, 50000, 12)
    c = grid.run(p, 0, 50000, 12).counter("crossings")
    assert c == int(rec[:, 2].sum())


def test_packet_moments_are_pure_diagnostics(require_gpu):
    """packet_moments = 0 (the CLI / bench setting) transports the same packets: every
    detector plane the reference writes, the counters and the fluxes are identical; only
    the packet-level moment planes 12-15 and totals[4:8] stay empty."""
    atm = synthetic.make_config("ray3d", nr=10, ntheta=6, nphi=8)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    from artes_amd.engine import Grid

    grid = Grid(atm, device=0)
    on = grid.run(driver.run_params(cfg, det, 0, cell_depth=-1, packet_moments=True), 0, 200000, 5)
    off = grid.run(driver.run_params(cfg, det, 0, cell_depth=-1, packet_moments=False), 0, 200000, 5)
    np.testing.assert_array_equal(on.counters, off.counters)
    np.testing.assert_allclose(off.det[:3], on.det[:3], rtol=1e-9, atol=1e-300)
    assert np.all(off.det[3] == 0) and on.det[3].sum() > 0
    np.testing.assert_allclose(off.totals[:4], on.totals[:4], rtol=1e-9)
    assert np.all(off.totals[4:8] == 0) and on.totals[4] > 0


def test_kernel_times_profiling(require_gpu):
    atm, grid, p = _setup()
    assert grid.kernel_times()["trace"] == (0.0, 0)          # profiling off: nothing recorded
    grid.set_profiling(True)
    grid.run(p, 0, 10**6, 1)
    kt = grid.kernel_times()
    assert kt["trace"][1] >= 2 and kt["trace"][0] > 0.0
    assert kt["event"][1] == kt["trace"][1] and kt["emit"][1] == kt["trace"][1] + 1
    total = sum(ms for ms, _ in kt.values())
    assert total <= grid.last_kernel_ms() * 1.05 + 0.5
    assert grid.kernel_times()["trace"] == (0.0, 0)          # reset after reading
    grid.set_tuning(engine="persistent")
    grid.run(p, 0, 10**5, 1)
    grid.set_tuning(engine=None)
    kt = grid.kernel_times()
    assert kt["persistent"][1] == 1 and kt["trace"][1] == 0


def test_unsupported_options_fail_loudly(require_gpu):
    from artes_amd.engine import EngineError

    atm, grid, p = _setup(nr=4, ntheta=4, nphi=4)
    p.photon_source = 2
    with pytest.raises(EngineError, match="planet"):
        grid.run(p, 0, 10, 1)
    p.photon_source = 1
    p.wl_index = 3
    with pytest.raises(EngineError, match="wl_index"):
        grid.run(p, 0, 10, 1)


def test_zero_and_tiny_runs(require_gpu):
    atm, grid, p = _setup("iso")
    r0 = grid.run(p, 0, 0, 1)
    assert r0.det.sum() == 0.0 and r0.counters.sum() == 0
    r1 = grid.run(p, 0, 1, 1)
    assert r1.counter("packets") == 1
    r7 = grid.run(p, 5, 7, 1)
    assert r7.counter("packets") == 7


def test_reused_pool_gives_fresh_results(require_gpu):
    """A grid's packet pool outlives its calls, and k_init no longer rewrites the slot records
    (kernel_event.hpp, k_init / k_emit: a fresh slot is known from its emit entry alone): a
    call after larger and smaller ones on the same grid gives the counters of a fresh grid
    and its detector to summation order."""
    atm, grid, p = _setup("ray3d", nr=10, ntheta=6, nphi=8)
    grid.run(p, 0, 200000, 11)
    grid.run(p, 3, 5000, 12)
    again = grid.run(p, 100, 60000, 13)
    grid.close()
    atm, fresh_grid, p = _setup("ray3d", nr=10, ntheta=6, nphi=8)
    fresh = fresh_grid.run(p, 100, 60000, 13)
    fresh_grid.close()
    np.testing.assert_array_equal(again.counters, fresh.counters)
    np.testing.assert_allclose(again.det, fresh.det, rtol=1e-9, atol=1e-300)
    np.testing.assert_array_equal(again.err, fresh.err)


def test_bench_line_contract(require_gpu):
    """bench.py (the driver's measurement) prints one JSON line with the contract's fields,
    on a small packet count (a subprocess: the bench owns its process)."""
    import json
    import subprocess
    import sys

    from conftest import ROOT

    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--packets", "2e6", "--steps", "2", "--warmup", "1",
                          "--no-cpu-baseline", "--no-variants", "--no-parity"],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    assert r["events_per_packet"]["crossings"] > 50 and d["errors"] == {}


def test_tuning_keys_are_checked(require_gpu):
    """artes_set_tuning: unknown keys and out-of-range values fail with -22 ("steps"
    other than 4 / 8 used to map silently to 8; the fine-grid kernel has 10 steps since round 6); -1
    restores a default."""
    from artes_amd.engine import EngineError

    atm, grid, p = _setup(nr=8, ntheta=8, nphi=8)
    for bad in (dict(steps=2), dict(steps=6), dict(steps=8), dict(batch_min=0), dict(event_block=512), dict(wpe=5), dict(nosuchkey=1)):
        with pytest.raises(EngineError):
            grid.set_tuning(**bad)
    assert grid.tuning() == {}
    grid.set_tuning(steps=4)
    grid.run(p, 0, 10**4, 1)
    assert grid.last_launch().startswith("k_trace<1,0,4,0,4>")
    grid.set_tuning(steps=None)
    assert grid.tuning() == {}
    grid.run(p, 0, 10**4, 1)
    assert grid.last_launch().startswith("k_trace<1,0,4,0,4>")   # (512 cells: a coarse grid)
    _, g1, p1 = _setup("hg")
    with pytest.raises(EngineError, match="radial-only"):
        g1.set_tuning(steps=4)


def test_production_library_ignores_environment(require_gpu):
    """The production library reads no ARTES_* variable: a child process with
    ARTES_ENGINE=persistent ARTES_STEPS=4 ARTES_POOL=3000 transports exactly what a clean one
    does, with the default kernels."""
    import json
    import subprocess
    import sys

    from conftest import ROOT

    script = (
        "import json, sys; sys.path.insert(0, %r)\n"
        "from artes_amd import driver, synthetic\n"
        "from artes_amd.engine import Grid\n"
        "atm = synthetic.make_config('ray3d', nr=16, ntheta=16, nphi=16)\n"
        "cfg = driver.default_config(); det = driver.detector_geometry(cfg, float(atm['radial'][-1]))\n"
        "g = Grid(atm, 0); p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))\n"
        "r = g.run(p, 0, 100000, 3)\n"
        "print(json.dumps(dict(l=g.last_launch(), c=[int(x) for x in r.counters], d=float(r.det[0].sum()), t=g.tuning())))\n"
    ) % ROOT
    outs = []
    for extra in ({}, dict(ARTES_ENGINE="persistent", ARTES_STEPS="4", ARTES_POOL="3000", ARTES_REFILL="1")):
        env = {k: v for k, v in os.environ.items() if not k.startswith("ARTES_")}
        env.update(extra)
        out = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-2000:]
        outs.append(json.loads(out.stdout.strip().splitlines()[-1]))
    # (the detector sums are FP64 atomics: their order, and so their last bits, varies run to run)
    d0, d1 = outs[0].pop("d"), outs[1].pop("d")
    assert abs(d0 - d1) <= 1e-12 * abs(d0)
    assert outs[0] == outs[1]
    assert outs[0]["l"] == "k_trace<1,0,4,0,10> k_event<1,1,0,768,0>" and outs[0]["t"] == {}

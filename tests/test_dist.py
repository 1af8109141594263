"""Multi-rank packet sharding + detector reduction, world_size 2 on gloo (CPU).

The per-rank transport here is the CPU oracle (test infrastructure), injected into the
product's sharding/reduction code (artes_amd.dist), which is what runs on RCCL on GPUs."""

import os
import subprocess
import sys

import numpy as np

from artes_amd import dist
from conftest import ROOT

WORKER = r'''
import os, sys
sys.path.insert(0, {root!r})
import numpy as np
import torch.distributed as tdist
from artes_amd import dist, driver, synthetic
from artes_amd.engine import RunResult
from oracle.oracle import OracleGrid

r = dist.init()   # backend from ARTES_DIST_BACKEND (the one-GPU rehearsal's switch)
atm = synthetic.make_config("ray3d", nr=6, ntheta=4, nphi=6)
cfg = driver.default_config()
det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
g = OracleGrid(atm)
p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))

def transport(first, n, seed):
    d, t, c, e, fg, ft = g.run_flow(p, first, n, seed, threads=2)
    return RunResult(d, t, c, e, fg, ft)

res = dist.run_sharded(transport, 30001, 99, r)
seed = dist.broadcast_int((2**62 + 12345) if r.rank == 0 else 777, r)   # the CLI's clock seed
open({out!r}.replace("det2.npy", "seed%d.txt" % r.rank), "w").write(str(seed))
# an unsharded call (world 1) inside this 2-rank group: not reduced (ADVICE r05)
solo = dist.run_sharded(transport, 5000, 7, dist.Rank(r.rank, 1, r.local_rank))
try:
    dist.reduces(3)
    mismatch = "accepted"
except RuntimeError:
    mismatch = "refused"
if r.rank == 0:
    np.save({out!r}.replace(".npy", "_solo.npy"), solo.det)
    open({out!r}.replace("det2.npy", "mismatch.txt"), "w").write(mismatch)
    open({out!r}.replace("det2.npy", "backend.txt"), "w").write(tdist.get_backend())
    np.save({out!r}, res.det)
    np.save({out!r}.replace(".npy", "_cnt.npy"), res.counters)
    np.save({out!r}.replace(".npy", "_flow.npy"), res.flow_global)
    np.save({out!r}.replace(".npy", "_lat.npy"), res.flow_latitudinal)
tdist.barrier()
tdist.destroy_process_group()
'''


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 10**9 + 3):
        for w in (1, 2, 3, 8):
            parts = [dist.shard(n, k, w) for k in range(w)]
            assert sum(c for _, c in parts) == n
            assert all(parts[k][0] + parts[k][1] == parts[k + 1][0] for k in range(w - 1))


def test_two_rank_gloo_equals_single_process(tmp_path):
    out = str(tmp_path / "det2.npy")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, out=out))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29633", WORLD_SIZE="2", ARTES_DIST_BACKEND="gloo")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(k), LOCAL_RANK=str(k)))
             for k in range(2)]
    for pr in procs:
        assert pr.wait(timeout=300) == 0
    assert open(str(tmp_path / "backend.txt")).read() == "gloo"
    assert [int(open(str(tmp_path / f"seed{k}.txt")).read()) for k in range(2)] == [2**62 + 12345] * 2
    det2 = np.load(out)
    cnt2 = np.load(out.replace(".npy", "_cnt.npy"))

    from artes_amd import driver, synthetic
    from oracle.oracle import OracleGrid

    atm = synthetic.make_config("ray3d", nr=6, ntheta=4, nphi=6)
    cfg = driver.default_config()
    det = driver.detector_geometry(cfg, float(atm["radial"][-1]))
    g = OracleGrid(atm)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0))
    d1, _, c1, _, fg1, ft1 = g.run_flow(p, 0, 30001, 99, threads=4)
    np.testing.assert_allclose(det2, d1, rtol=1e-11, atol=1e-300)
    np.testing.assert_array_equal(cnt2, c1)
    # the flow diagnostics are summed over the ranks too
    np.testing.assert_allclose(np.load(out.replace(".npy", "_flow.npy")), fg1, rtol=1e-10, atol=1e-12 * np.abs(fg1).max())
    np.testing.assert_allclose(np.load(out.replace(".npy", "_lat.npy")), ft1, rtol=1e-11, atol=1e-300)
    # a world-1 call inside the group transports all its packets on each rank and is not summed
    d_solo = g.run_flow(p, 0, 5000, 7, threads=4)[0]
    np.testing.assert_allclose(np.load(out.replace(".npy", "_solo.npy")), d_solo, rtol=1e-11, atol=1e-300)
    assert open(str(tmp_path / "mismatch.txt")).read() == "refused"


def test_device_of_is_local_rank_modulo_visible_devices(monkeypatch):
    """One rank-to-device rule for the CLI, the bench and the RCCL device (dist.device_of):
    local_rank modulo the visible devices, so ranks sharing one card (the gloo rehearsal on a
    one-GPU box) and launchers that show each rank one GPU both map inside [0, count)."""
    import torch

    for count, local, want in ((8, 3, 3), (1, 1, 0), (1, 7, 0), (0, 5, 0), (2, 5, 1)):
        monkeypatch.setattr(torch.cuda, "device_count", lambda c=count: c)
        assert dist.device_of(dist.Rank(rank=local, world=8, local_rank=local)) == want


def test_bench_host_cores_reports_the_usable_count():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    c = bench.host_cores()
    assert c["affinity"] == len(os.sched_getaffinity(0)) and 1 <= c["usable"] <= c["affinity"] <= c["visible"]

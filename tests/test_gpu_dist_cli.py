"""The drop-in CLI under two ranks ON THE HIP ENGINE (gloo process group, both ranks on the
one card of the GPU box) against one process.

``runner.run`` with its default transport, as ``python -m artes_amd`` / ``./bin/ARTES``
run it under ``torch.distributed.run``: every rank opens the engine on ``dist.device_of``
(``local_rank`` modulo the visible devices, so rank 1 of a one-GPU box uses device 0),
transports its shard of every call's global packet ids, the sums are all-reduced
(``dist.run_sharded``) and rank 0 writes the output tree -- the reference's thread
reduction (``ARTES.f90:534-546``, ``957-975``) across processes.  The RNG is keyed by the
global packet id, so the union of the shards is the one-process run: the files that do not
depend on the packet sums are byte-identical, and the sums agree to their summation order
(the engine's FP64 detector atomics already reorder them between two one-process runs)."""

import os
import subprocess
import sys

import numpy as np
import pytest

from artes_amd import atmosphere, fitsio, runner, synthetic
from conftest import ROOT
from test_dist_cli import ARTES_IN, EXACT, _files, _rows

pytestmark = pytest.mark.gpu

WORKER = r'''
import sys
sys.path.insert(0, {root!r})
import torch.distributed as tdist
from artes_amd import runner
for mode, n in (("imaging_mono", "{n_img}"), ("spectrum", "{n_spec}")):
    assert runner.run(["atm_" + mode, n, "-o", "r2_" + mode, "-k", "photon:fstop=2d-5", "--seed", "77"],
                      root={root_dir!r}) == 0
    tdist.barrier()
tdist.destroy_process_group()
'''

N_IMG, N_SPEC = "2e6", "1e6"


def test_cli_two_ranks_on_hip_engine_equals_one(tmp_path, require_gpu):
    for mode in ("imaging_mono", "spectrum"):
        d = tmp_path / "input" / f"atm_{mode}"
        d.mkdir(parents=True)
        (d / "artes.in").write_text(ARTES_IN.format(mode=mode))
        kw = dict(nr=8, ntheta=6, nphi=8) if mode == "imaging_mono" else dict(nr=8, wavelength=(0.5, 0.7, 0.9))
        atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"),
                                         synthetic.make_config("ray3d" if mode == "imaging_mono" else "hg", **kw))
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, root_dir=str(tmp_path), n_img=N_IMG, n_spec=N_SPEC))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29653", WORLD_SIZE="2", ARTES_DIST_BACKEND="gloo")
    env.pop("ARTES_LIB_PATH", None)
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(k), LOCAL_RANK=str(k)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for k in range(2)]
    logs = []
    for pr in procs:
        out, _ = pr.communicate(timeout=240)
        logs.append(out)
        assert pr.returncode == 0, out[-3000:]
    assert "imaging_mono, 2000000 packets" in logs[0]

    for mode in ("imaging_mono", "spectrum"):
        n = N_IMG if mode == "imaging_mono" else N_SPEC
        assert runner.run([f"atm_{mode}", n, "-o", f"r1_{mode}", "-k", "photon:fstop=2d-5", "--seed", "77"],
                          root=str(tmp_path)) == 0
        one, two = tmp_path / "output" / f"r1_{mode}", tmp_path / "output" / f"r2_{mode}"
        assert _files(one) == _files(two)
        for f in EXACT:
            if (one / f).exists():
                assert (one / f).read_bytes() == (two / f).read_bytes(), f
        assert (one / "error.log").read_text() == ""
        if mode == "imaging_mono":
            s1, s2 = (fitsio.read(x / "output" / "stokes.fits")[0].data for x in (one, two))
            assert s1[0].sum() > 0
            np.testing.assert_allclose(s2, s1, rtol=1e-11, atol=1e-11 * np.abs(s1).max())
            e1, e2 = (fitsio.read(x / "output" / "error.fits")[0].data[:4] for x in (one, two))
            np.testing.assert_allclose(e2, e1, rtol=1e-7, atol=1e-7 * np.abs(e1).max())
            p1, p2 = _rows(one / "output/photometry.dat"), _rows(two / "output/photometry.dat")
        else:
            p1, p2 = _rows(one / "output/spectrum.dat"), _rows(two / "output/spectrum.dat")
            assert p1.shape == (3, 5) and np.all(p1[:, 1] > 0)
        # column 0 is the wavelength; the flux columns (Stokes I, Q, U, V and, in photometry.dat,
        # their sigmas) against Stokes I's scale, since Q and U sums cancel towards zero
        np.testing.assert_array_equal(p2[:, 0], p1[:, 0])
        np.testing.assert_allclose(p2[:, 1:], p1[:, 1:], rtol=1e-9, atol=1e-11 * np.abs(p1[:, 1]).max())


RCCL_WORKER = r'''
import json, sys
sys.path.insert(0, {root!r})
import torch.distributed as tdist
from artes_amd import dist, runner
for mode, n in (("imaging_mono", "{n_img}"), ("spectrum", "{n_spec}")):
    assert runner.run(["atm_" + mode, n, "-o", "rc_" + mode, "-k", "photon:fstop=2d-5", "--seed", "77"],
                      root={root_dir!r}) == 0
r = dist.env_rank()
v = (0x1234ABCD << 32) | 0x0F0F0F0F
b = dist.broadcast_int(v, r)
print(json.dumps(dict(backend=tdist.get_backend(), world=tdist.get_world_size(), coll=dist.COLLECTIVES, bcast=b == v)))
tdist.destroy_process_group()
'''


def test_cli_rccl_one_rank_equals_plain(tmp_path, require_gpu):
    """The CLI's RCCL reduction path: a fresh process with a one-rank `nccl`
    process group (ARTES_DIST_FORCE=1, ARTES_DIST_BACKEND=nccl, set up before any GPU call)
    runs ``runner.run`` on imaging_mono and a 3-wavelength spectrum; every engine call's sums
    then travel through the GPU in ``dist.allreduce_numpy``'s device branch, and
    ``dist.broadcast_int`` (the clock seed shared across ranks) rides on it.  The output
    trees equal the plain one-process run's (ARTES.f90:534-546, 957-975)."""
    import json

    for mode in ("imaging_mono", "spectrum"):
        d = tmp_path / "input" / f"atm_{mode}"
        d.mkdir(parents=True)
        (d / "artes.in").write_text(ARTES_IN.format(mode=mode))
        kw = dict(nr=8, ntheta=6, nphi=8) if mode == "imaging_mono" else dict(nr=8, wavelength=(0.5, 0.7, 0.9))
        atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"),
                                         synthetic.make_config("ray3d" if mode == "imaging_mono" else "hg", **kw))
    script = tmp_path / "rccl_worker.py"
    script.write_text(RCCL_WORKER.format(root=ROOT, root_dir=str(tmp_path), n_img=N_IMG, n_spec=N_SPEC))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29657", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               ARTES_DIST_FORCE="1", ARTES_DIST_BACKEND="nccl")
    env.pop("ARTES_LIB_PATH", None)
    out = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    info = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert info["backend"] == "nccl" and info["world"] == 1 and info["bcast"], info
    # one device all-reduce per engine call: 1 imaging call + 3 wavelengths, + the broadcast
    assert info["coll"]["device"] == 1 + 3 + 1 and info["coll"]["host"] == 0, info

    for mode in ("imaging_mono", "spectrum"):
        n = N_IMG if mode == "imaging_mono" else N_SPEC
        assert runner.run([f"atm_{mode}", n, "-o", f"p1_{mode}", "-k", "photon:fstop=2d-5", "--seed", "77"],
                          root=str(tmp_path)) == 0
        one, rc = tmp_path / "output" / f"p1_{mode}", tmp_path / "output" / f"rc_{mode}"
        assert _files(one) == _files(rc)
        for f in EXACT:
            if (one / f).exists():
                assert (one / f).read_bytes() == (rc / f).read_bytes(), f
        if mode == "imaging_mono":
            s1, s2 = (fitsio.read(x / "output" / "stokes.fits")[0].data for x in (one, rc))
            assert s1[0].sum() > 0
            np.testing.assert_allclose(s2, s1, rtol=1e-11, atol=1e-11 * np.abs(s1).max())
            p1, p2 = _rows(one / "output/photometry.dat"), _rows(rc / "output/photometry.dat")
        else:
            p1, p2 = _rows(one / "output/spectrum.dat"), _rows(rc / "output/spectrum.dat")
            assert p1.shape == (3, 5)
        np.testing.assert_array_equal(p2[:, 0], p1[:, 0])
        np.testing.assert_allclose(p2[:, 1:], p1[:, 1:], rtol=1e-9, atol=1e-11 * np.abs(p1[:, 1]).max())

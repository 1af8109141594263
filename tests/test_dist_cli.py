"""The drop-in CLI (``runner.run``) under two ranks (gloo, CPU) against one process.

Every rank runs ``python -m artes_amd``'s code path with the same argv; rank k transports
its shard of every call's global packet ids, the sums of each call are all-reduced
(``dist.run_sharded``) and rank 0 writes the output tree -- the reference's thread
reduction (``ARTES.f90:534-546``, ``957-975``) across processes.  The per-rank transport
is the CPU oracle (test infrastructure), as in tests/test_dist.py.  Files that do not
depend on the packet sums are byte-identical to the single-process run's; the ones that
do agree to the summation order (1e-12 relative; error.fits's sigma, a difference of two
sums, to 1e-9)."""

import os
import subprocess
import sys

import numpy as np
import pytest

from artes_amd import atmosphere, fitsio, runner, synthetic
from conftest import ROOT

WORKER = r'''
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import torch.distributed as tdist
from artes_amd import runner
from test_cli import OracleTransport
for mode, n in (("imaging_mono", "3e4"), ("spectrum", "2e4")):
    assert runner.run(["atm_" + mode, n, "-o", "r2_" + mode, "-k", "photon:fstop=2d-5", "--seed", "77"],
                      root={root_dir!r}, transport_factory=OracleTransport) == 0
    tdist.barrier()
tdist.destroy_process_group()
'''

ARTES_IN = """* two-rank CLI test
photon:source=star
photon:fstop=1d-5
photon:minimum=1d-20
star:temperature=5800
star:radius=1
planet:orbit=5
detector:type={mode}
detector:theta=90
detector:phi=90
detector:pixel=25
detector:distance=10
"""

EXACT = ("error.log", "plot.dat", "input/artes.in", "input/atmosphere.fits", "output/normalization.dat",
         "output/cell_depth.dat", "output/optical_depth.dat")


def _rows(path):
    return np.array([[float(v) for v in l.split()] for l in open(path).read().splitlines() if l.strip() and "#" not in l])


def _files(d):
    return sorted(os.path.relpath(os.path.join(a, f), d) for a, _, fs in os.walk(d) for f in fs)


def test_cli_two_ranks_equals_one(tmp_path):
    for mode in ("imaging_mono", "spectrum"):
        d = tmp_path / "input" / f"atm_{mode}"
        d.mkdir(parents=True)
        (d / "artes.in").write_text(ARTES_IN.format(mode=mode))
        kw = dict(nr=6, ntheta=4, nphi=6) if mode == "imaging_mono" else dict(nr=6, wavelength=(0.5, 0.7, 0.9))
        atmosphere.write_atmosphere_fits(str(d / "atmosphere.fits"),
                                         synthetic.make_config("ray3d" if mode == "imaging_mono" else "hg", **kw))
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, tests=os.path.join(ROOT, "tests"), root_dir=str(tmp_path)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29651", WORLD_SIZE="2", ARTES_DIST_BACKEND="gloo")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(k), LOCAL_RANK=str(k)))
             for k in range(2)]
    for pr in procs:
        assert pr.wait(timeout=600) == 0
    from test_cli import OracleTransport

    for mode in ("imaging_mono", "spectrum"):
        assert runner.run([f"atm_{mode}", "3e4" if mode == "imaging_mono" else "2e4", "-o", f"r1_{mode}", "-k",
                           "photon:fstop=2d-5", "--seed", "77"], root=str(tmp_path),
                          transport_factory=OracleTransport) == 0
        one, two = tmp_path / "output" / f"r1_{mode}", tmp_path / "output" / f"r2_{mode}"
        assert _files(one) == _files(two)
        for f in EXACT:
            if (one / f).exists():
                assert (one / f).read_bytes() == (two / f).read_bytes(), f
        if mode == "imaging_mono":
            s1, s2 = (fitsio.read(x / "output" / "stokes.fits")[0].data for x in (one, two))
            np.testing.assert_allclose(s2, s1, rtol=1e-12, atol=1e-12 * np.abs(s1).max())
            e1, e2 = (fitsio.read(x / "output" / "error.fits")[0].data[:4] for x in (one, two))
            np.testing.assert_allclose(e2, e1, rtol=1e-9, atol=1e-9 * np.abs(e1).max())
            p1, p2 = _rows(one / "output/photometry.dat"), _rows(two / "output/photometry.dat")
            assert s1[0].sum() > 0
        else:
            p1, p2 = _rows(one / "output/spectrum.dat"), _rows(two / "output/spectrum.dat")
            assert p1.shape == (3, 5) and np.all(p1[:, 1] > 0)
        np.testing.assert_allclose(p2, p1, rtol=1e-12, atol=1e-12 * np.abs(p1).max())

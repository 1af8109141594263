"""End-to-end drop-in CLI throughput on the gas + Mie-cloud input (development tool).

Builds the configs[3]-shaped atmosphere (artes_amd.synthetic.make_cloudy, 3 wavelengths)
as input/<atm>/ in a scratch directory and times ``python -m artes_amd``-equivalent runs
(runner.run) in spectrum and phase mode, FITS reading and output writing included.
usage: python tools/cli_perf.py [packets per call]"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from artes_amd import driver, runner, synthetic  # noqa: E402

ARTES_IN = """photon:source=star
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
n = sys.argv[1] if len(sys.argv) > 1 else "1e8"
with tempfile.TemporaryDirectory() as root:
    d = os.path.join(root, "input", "cloudy")
    synthetic.make_cloudy(d)
    for mode, calls in (("spectrum", 3), ("phase", len(driver.phase_angles()))):
        open(os.path.join(d, "artes.in"), "w").write(ARTES_IN.format(mode=mode))
        t = time.perf_counter()
        rc = runner.run(["cloudy", n, "-o", f"perf_{mode}", "--seed", "7"], root=root)
        dt = time.perf_counter() - t
        total = float(n) * calls
        log = os.path.join(root, "output", f"perf_{mode}", "error.log")
        if os.path.exists(log):
            print(open(log).read().strip()[:2000], flush=True)
        print(f"{mode}: {calls} engine calls x {float(n):.0e} packets, {dt:.2f} s wall incl. I/O "
              f"-> {total / dt / 1e6:.1f} Mpackets/s (rc {rc})", flush=True)

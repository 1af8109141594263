"""Cost of the bench's per-launch HIP events (development tool): the bench step (the metric's 32^3
grid, 1e9 packets) timed with artes_set_profiling off and on, alternating.
usage: python tools/prof_overhead.py [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg = driver.default_config()
atm = synthetic.make_config("ray3d", ntheta=32, normalizer="simpson", share_matrix=True)
geom = driver.detector_geometry(cfg, float(atm["radial"][-1]))
g = Grid(atm, device=0)
p = driver.run_params(cfg, geom, 0, cell_depth=g.cell_depth(0), packet_moments=False)
det = torch.zeros(16 * geom.ny * geom.nx, dtype=torch.float64, device="cuda:0")
stream = torch.cuda.current_stream()
n = 10**9


def step(k):
    g.run_device(p, k * n, n, 1234, det.data_ptr(), 0, 0, 0, stream.cuda_stream)


g.set_profiling(True)
step(0)
torch.cuda.synchronize()
g.kernel_times()
k = 1
for r in range(rounds):
    for prof in (False, True):
        g.set_profiling(prof)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            step(k)
            k += 1
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 2 * 1e3
        g.kernel_times()
        print(f"profiling {'on ' if prof else 'off'}: {ms:.1f} ms per 1e9-packet step", flush=True)

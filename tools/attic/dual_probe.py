"""Two event engines on two HIP streams at once vs one (development tool).

Each k_trace launch ends in a tail of a few long traces; a second engine on its own
stream can fill the CUs the first one's tail leaves idle.  Host threads drive the two
grids (ctypes releases the GIL during artes_run_device).
usage: python tools/dual_probe.py [n_packets] [workload]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from artes_amd import driver, synthetic  # noqa: E402
from artes_amd.engine import Grid  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 4 * 10**8
name = sys.argv[2] if len(sys.argv) > 2 else "ray3d"
cfg = driver.default_config()
atm = synthetic.make_config(name, share_matrix=True)
det = driver.detector_geometry(cfg, atm["radial"][-1])


def bufs():
    f = dict(dtype=torch.float64, device="cuda:0")
    return torch.zeros(4, 4, 25, 25, **f), torch.zeros(8, **f)


def run_single(pool):
    os.environ["ARTES_POOL"] = str(pool)
    g = Grid(atm, 0)
    p = driver.run_params(cfg, det, 0, cell_depth=g.cell_depth(0), packet_moments=False)
    d, t = bufs()
    s = torch.cuda.Stream()
    g.run_device(p, 0, 10**6, 1, d.data_ptr(), t.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.run_device(p, 0, n, 2024, d.data_ptr(), t.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g.close()
    return dt, d[0, 0].sum().item()


def run_dual(pool, k=2):
    os.environ["ARTES_POOL"] = str(pool)
    gs = [Grid(atm, 0) for _ in range(k)]
    p = driver.run_params(cfg, det, 0, cell_depth=gs[0].cell_depth(0), packet_moments=False)
    bs = [bufs() for _ in range(k)]
    ss = [torch.cuda.Stream() for _ in range(k)]
    for g, (d, t), s in zip(gs, bs, ss):
        g.run_device(p, 0, 10**6, 1, d.data_ptr(), t.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    for d, t in bs:
        d.zero_()
    torch.cuda.synchronize()

    def work(i):
        g, (d, t), s = gs[i], bs[i], ss[i]
        g.run_device(p, i * (n // k), n // k, 2024, d.data_ptr(), t.data_ptr(), stream=s.cuda_stream)
        s.synchronize()

    th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot = sum(d[0, 0].sum().item() for d, _ in bs)
    for g in gs:
        g.close()
    return dt, tot


cus = torch.cuda.get_device_properties(0).multi_processor_count
full = cus * 65536
for label, fn in [("single full", lambda: run_single(full)), ("dual half", lambda: run_dual(full // 2)),
                  ("dual full", lambda: run_dual(full)), ("single full", lambda: run_single(full)),
                  ("quad quarter", lambda: run_dual(full // 4, 4))]:
    dt, tot = fn()
    print(f"{name} {label}: {n / dt / 1e6:.1f} Mpackets/s  ({dt * 1e3:.0f} ms, I sum {tot:.6e})", flush=True)

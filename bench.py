#!/usr/bin/env python3
"""Benchmark: photon packets per second on the BASELINE.json headline configuration.

Workload: the metric's "32^3 grid" (BASELINE.json `metric`) with BASELINE configs[2]'s
physics: Rayleigh-polarised atmosphere (full 16-element Mueller matrix), 32 x 32 x 32
(r, theta, phi) cells, one wavelength, star source, imaging_mono 25 x 25 detector at
theta = phi = 90 deg, radial tau = 1, albedo 1.  configs[2]'s own 32 x 16 x 32 grid is
reported beside it (one untimed step, `configs2_32x16x32`), and the Stokes-I parity step
runs on that grid (the frozen reference runs are of it).
One step = one `radiative_transfer` call (ARTES.f90:518-1006) of `--packets` packets
per GPU (default 1e9 = the config's packet count), followed by the RCCL sum-reduce of
the detector over ranks.  Weak scaling: every GPU transports `--packets` per step.

Run:   python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
           --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
Prints ONE JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# canonical algorithmic bytes per packet: 8 B of kappa per crossing,
# 304 B per scatter (albedo 8 + p1j 32 + two 16-element f64 rows 256 + ...), 352 B per
# peel (two matrix rows 256 + 12-value detector read-modify-write 96)
B_PER_CROSSING, B_PER_SCATTER, B_PER_PEEL = 8.0, 304.0, 352.0
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)


def host_cores() -> dict:
    """The host cores this process may use: the affinity mask, capped by the cgroup's CPU
    quota when one is set (a container's share of a larger machine), and the machine's count."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:                                       # cgroup v2
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        try:                                   # cgroup v1
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            if q > 0:
                quota = q / float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        except (OSError, ValueError):
            pass
    usable = affinity if quota is None else max(1, min(affinity, int(math.ceil(quota))))
    return {"visible": os.cpu_count() or 1, "affinity": affinity,
            "cgroup_quota": None if quota is None else round(quota, 2), "usable": usable}


def cpu_baseline(atm, params, budget_s: float = 15.0, single_s: float = 4.0) -> dict:
    """The CPU oracle (C restatement of the reference packet loop, OpenMP) on every host core
    this process may use (``ARTES_CPU_THREADS`` overrides), plus a one-thread rate: DESIGN.md
    §6 calibrates the port against the reference per core (1.2-1.5x)."""
    from oracle import oracle

    cores = host_cores()
    threads = int(os.environ.get("ARTES_CPU_THREADS", cores["usable"]))
    g = oracle.OracleGrid(atm)

    def rate(first, threads, budget):
        probe = 2000 * threads
        t0 = time.perf_counter()
        g.run(params, first, probe, 99, threads=threads)
        r = probe / max(time.perf_counter() - t0, 1e-6)
        n = int(min(max(r * budget, 2e4), 5e7))
        t0 = time.perf_counter()
        g.run(params, first + probe, n, 99, threads=threads)
        dt = time.perf_counter() - t0
        return n, dt

    n, dt = rate(10**12, threads, budget_s)
    n1, dt1 = rate(2 * 10**12, 1, single_s)
    return {"value": round(n / dt / 1e6, 4), "unit": "Mphotons/s", "cores": threads, "kind": "port",
            "cores_visible": cores["visible"], "cores_affinity": cores["affinity"],
            "cgroup_cpu_quota": cores["cgroup_quota"],
            "one_thread": {"value": round(n1 / dt1 / 1e6, 5), "unit": "Mphotons/s", "packets": n1, "seconds": round(dt1, 2)},
            "sample": f"{n} packets of the same ray3d workload (oracle/artes_oracle.c, {threads} OpenMP threads, {dt:.1f} s; "
                      f"threads = the affinity mask's cores capped by the cgroup CPU quota)"}


def _md5(path: str) -> str | None:
    import hashlib

    try:
        return hashlib.md5(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


def main() -> int:
    # stdout carries exactly one JSON line (rank 0): libraries that print to the process's
    # descriptor 1 -- RCCL writes its version banner there when a communicator starts -- are
    # pointed at stderr, and the line is written to the saved descriptor
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--packets", type=float, default=1e9, help="packets per GPU per step")
    ap.add_argument("--seed", type=int, default=20171015)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the untimed parity step (profiling passes)")
    ap.add_argument("--no-variants", action="store_true", help="skip the untimed configs[2] (32x16x32) leg (profiling passes)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r06", "pmc_summary.json"))
    ap.add_argument("--sq-json", default=os.path.join(ROOT, "profiles", "r06", "pmc_sq_summary.json"))
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="an artes_set_tuning override of the bench grid (measurements only, e.g. det_ordered=1; "
                         "reported under engine.tuning)")
    args = ap.parse_args()

    import numpy as np
    import torch

    from artes_amd import dist, driver, stats, synthetic
    from artes_amd.engine import Grid

    r = dist.init()
    world = r.world
    # one GPU per rank; more ranks than devices only in a gloo rehearsal (ARTES_DIST_BACKEND=gloo),
    # since RCCL refuses two ranks on one device
    dev = dist.device_of(r)
    torch.cuda.set_device(dev)
    per_gpu = int(args.packets)

    cfg = driver.default_config()
    # the headline grid: the metric's 32^3 cells, configs[2]'s physics (the survey's inputs
    # for the frozen reference runs, tests/golden/README.md, with 32 theta cells)
    atm = synthetic.make_config("ray3d", ntheta=32, normalizer="simpson", share_matrix=True)
    rtop = float(atm["radial"][-1])
    det_geom = driver.detector_geometry(cfg, rtop)
    grid = Grid(atm, device=dev)
    for kv in args.tune:
        k, v = kv.split("=", 1)
        grid.set_tuning(**{k: int(v)})
    # the timed steps run the drop-in's production configuration: no packet-level moments
    # (the reference has none); the parity check below reruns one step with them
    params = driver.run_params(cfg, det_geom, 0, cell_depth=grid.cell_depth(0), packet_moments=False)
    ny, nx = det_geom.ny, det_geom.nx

    f64 = dict(dtype=torch.float64, device=f"cuda:{dev}")
    # one flat float64 buffer holds everything the ranks exchange, so a step issues ONE sum
    # all_reduce: the detector [4][4][ny][nx], sum T^2 per Stokes + the two
    # thermal fluxes (include/artes_amd.h), the counters and the error-code counts (the
    # engine writes those as uint64 into the int64 tensors; they are converted to float64,
    # exact below 2^53, before the reduce)
    n_det = 16 * ny * nx
    flat = torch.zeros(n_det + 6 + 8 + 64, **f64)
    det = flat[:n_det].view(4, 4, ny, nx)
    tot2 = flat[n_det:n_det + 6]
    cnt = torch.zeros(8, dtype=torch.int64, device=f"cuda:{dev}")
    err = torch.zeros(64, dtype=torch.int64, device=f"cuda:{dev}")
    stream = torch.cuda.current_stream()
    backend = None
    # the collective path (the step's all_reduce, the max-over-ranks timing, the barriers) runs
    # with more than one rank, or at one rank when ARTES_DIST_FORCE=1 initialised a process
    # group anyway (dist.init): RCCL's one-rank rehearsal of that path on a one-GPU box
    import torch.distributed as tdist
    coll = world > 1 or (tdist.is_available() and tdist.is_initialized())
    if coll:
        backend = tdist.get_backend()

    def step(k: int):
        flat.zero_(); cnt.zero_(); err.zero_()
        first = (k * world + r.rank) * per_gpu
        grid.run_device(params, first, per_gpu, args.seed, det.data_ptr(), tot2.data_ptr(), cnt.data_ptr(),
                        err.data_ptr(), stream.cuda_stream)
        if coll:
            flat[n_det + 6:n_det + 14].copy_(cnt)
            flat[n_det + 14:].copy_(err)
            tdist.all_reduce(flat)

    def counts():
        """(counters, error codes) of the last step, summed over ranks."""
        if coll:
            return (flat[n_det + 6:n_det + 14].cpu().numpy().astype(np.float64),
                    np.rint(flat[n_det + 14:].cpu().numpy()).astype(np.int64))
        return cnt.cpu().numpy().astype(np.float64), err.cpu().numpy()

    def barrier():
        torch.cuda.synchronize()
        if coll:
            tdist.barrier()
        torch.cuda.synchronize()

    # warmup; the last warmup step runs with the per-launch HIP events on, so the timed
    # region records events that already exist (no hipEventCreate inside it)
    for k in range(args.warmup):
        grid.set_profiling(k == args.warmup - 1)
        step(k)
    barrier()
    grid.kernel_times()            # drop the warmup's launches
    grid.set_profiling(True)       # HIP events around every transport launch (per-kernel durations)
    ev = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step(args.warmup + k)          # the transport kernels run on `stream`; the all_reduce follows
        e1.record(stream)
        ev.append((e0, e1))
    barrier()
    elapsed = time.perf_counter() - t0
    # step durations (HIP events on the launch stream: run_device + the RCCL reduce) and the
    # per-kernel launch durations (the library's events, same stream) over the timed region
    step_ms = [a.elapsed_time(b) for a, b in ev]
    ktimes = grid.kernel_times()   # {class: (summed ms over the timed steps, launches)}
    grid.set_profiling(False)
    # what ran: the library build, the kernel instantiations of the timed calls and the schedule
    # overrides of the handle (none in production: the library reads no environment variable)
    from artes_amd import engine as _engine
    engine_info = {"build": _engine.lib().artes_build_info().decode(), "kernels": grid.last_launch(),
                   "tuning": grid.tuning(), "lib_md5": _md5(_engine.LIB_PATH)}
    if coll:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    cnt_h, err_h = counts()
    if r.rank != 0:
        if coll:
            tdist.barrier()
        return 0

    total_packets = per_gpu * world * args.steps
    value = total_packets / elapsed / 1e6
    n_step = per_gpu * world
    C = cnt_h[0] / n_step
    S = cnt_h[1] / n_step
    P = cnt_h[2] / n_step
    b_alg = B_PER_CROSSING * C + B_PER_SCATTER * S + B_PER_PEEL * P
    kernels = {k: {"ms_per_step": round(ms / args.steps, 3), "launches_per_step": round(n / args.steps, 1),
                   "avg_launch_ms": round(ms / n, 4) if n else None}
               for k, (ms, n) in ktimes.items() if n}
    # the whole transport of one step is a pipeline of launches (k_trace / k_event / k_emit
    # per iteration): B_alg over the summed launch durations
    k_ms = sum(ms for ms, _ in ktimes.values()) / args.steps
    pipeline_gbs = b_alg * per_gpu / (k_ms * 1e-3) / 1e9
    # the roofline is quoted for the DOMINANT kernel, k_trace: its share of B_alg (the kappa
    # gather of every crossing, 8 B, and the albedo read at every interaction, 8 B) times the
    # packets one launch carries, over its average launch duration (HIP events, timed region)
    t_ms, t_n = ktimes.get("trace", (0.0, 0))
    trace_bpp = B_PER_CROSSING * C + 8.0 * S
    per_launch = trace_bpp * per_gpu * args.steps / t_n if t_n else 0.0
    avg_ms = t_ms / t_n if t_n else float("nan")
    achieved = per_launch / (avg_ms * 1e-3) / 1e9 if t_n else 0.0
    # HBM traffic of k_trace from the PMC passes (tools/gpu_round.sh): only when they profiled
    # THIS build of the library (its md5 is recorded in the summary), else null
    traffic, traffic_src, limiter = None, None, None
    lib_md5 = _md5(os.path.join(ROOT, "artes_amd", "lib", "libartes_hip.so"))
    for path, key in ((args.pmc_json, "pmc"), (args.sq_json, "sq")):
        try:
            prof = json.load(open(path))
        except Exception:
            continue
        if prof.get("lib_md5") != lib_md5:
            continue
        kt = {k: v for k, v in prof.get("kernels", {}).items() if k.startswith("k_trace")}
        if key == "pmc" and kt:
            bpp = next(iter(kt.values())).get("fabric_bytes_per_packet")
            if bpp:
                traffic = round(bpp * per_gpu * args.steps / t_n) if t_n else None
                traffic_src = os.path.relpath(path, ROOT)
        if key == "sq" and kt:
            limiter = {"source": os.path.relpath(path, ROOT), **next(iter(kt.values()))}
            if "valu_busy" in limiter and "salu_busy" in limiter:
                # issue-side limiter: the VALU and SALU wave-instructions' issue cycles (4 per
                # wave64 instruction on a SIMD) over the SIMD cycles available to the kernel
                limiter["issue_frac"] = round(limiter["valu_busy"] + limiter["salu_busy"], 4)
    err_rate = {str(i): {"count": int(e), "per_packet": float(e) / n_step} for i, e in enumerate(err_h) if e}

    # configs[2]'s own grid, 32 x 16 x 32 (r, theta, phi): one untimed step of the same packet
    # count on rank 0 at N = 1, and (on rank 0 at any N, the other ranks waiting at the final
    # barrier) the Stokes-I parity step (the frozen reference runs, tests/golden, are of this
    # grid): one more step, untimed, with the packet-level moments the honest per-pixel
    # errors need, against the reference's 1e6-packet image
    parity, cfg2 = None, None
    ref_dir = os.path.join(ROOT, "tests", "golden", "reference_runs", "t_ray3d_ARTES_det_1e6")
    if not ((args.no_variants or world > 1) and args.no_parity):
        atm2 = synthetic.make_config("ray3d", normalizer="simpson", share_matrix=True)
        g2 = Grid(atm2, device=dev)
        d2 = driver.detector_geometry(cfg, float(atm2["radial"][-1]))
        p2 = driver.run_params(cfg, d2, 0, cell_depth=g2.cell_depth(0), packet_moments=False)
        if world == 1 and not args.no_variants:
            det.zero_(); tot2.zero_(); cnt.zero_()
            g2.run_device(p2, 0, 10**7, args.seed, det.data_ptr(), tot2.data_ptr(), 0, 0, stream.cuda_stream)
            torch.cuda.synchronize()
            cnt.zero_()
            t2 = time.perf_counter()
            g2.run_device(p2, 0, per_gpu, args.seed, det.data_ptr(), tot2.data_ptr(), cnt.data_ptr(), 0, stream.cuda_stream)
            torch.cuda.synchronize()
            dt2 = time.perf_counter() - t2
            c2 = cnt.cpu().numpy().astype(np.float64) / per_gpu
            cfg2 = {"grid": "32x16x32 (r,theta,phi), BASELINE configs[2]", "value": round(per_gpu / dt2 / 1e6, 3),
                    "unit": "Mphotons/s", "packets": per_gpu, "ms": round(dt2 * 1e3, 3),
                    "events_per_packet": {"crossings": round(c2[0], 3), "scatters": round(c2[1], 4)},
                    "sample": "one untimed-region step on rank 0, same workload otherwise"}
        if os.path.isdir(ref_dir) and not args.no_parity:
            check = driver.run_params(cfg, d2, 0, cell_depth=g2.cell_depth(0), packet_moments=True)
            det.zero_(); tot2.zero_()
            g2.run_device(check, 0, per_gpu, args.seed + 1, det.data_ptr(), tot2.data_ptr(), 0, 0, stream.cuda_stream)
            torch.cuda.synchronize()
            raw = det.cpu().numpy()
            r2 = float(atm2["radial"][-1])
            E = driver.package_energy(cfg, float(atm2["wavelength"][0]) * 1e-6, r2, per_gpu, d2.det_phi)
            cmp = stats.compare_to_reference(raw, per_gpu, E, d2.pixel_scale, stats.load_reference_run(ref_dir), 10**6)
            ph = driver.photometry(driver.scale_detector(raw[:3], E))
            ref_ph = stats.load_reference_run(ref_dir)["photometry"]
            parity = {"stokes_I_rms_z": round(cmp["rms_z"], 4), "stokes_I_mean_z": round(cmp["mean_z"], 4),
                      "pixels": cmp["n_pixels"], "I_total": ph[0] * 1e-6, "I_total_reference": float(ref_ph[1]),
                      "reference": "tests/golden/reference_runs/t_ray3d_ARTES_det_1e6 (1e6 packets, 32x16x32 grid)",
                      "sample": f"{per_gpu} packets on rank 0 on the configs[2] grid, untimed, packet moments on"}
        g2.close()

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(atm, params)

    out = {
        "metric": json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"],
        "value": round(value, 3),
        "unit": "Mphotons/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (uniform Rayleigh atmosphere, generated in-process; no checkpoint/dataset)",
        "config": {"workload": "metric's 32^3 grid with BASELINE configs[2]'s physics: Rayleigh 16-element Mueller, "
                               "32x32x32 (r,theta,phi), 1 wavelength, star source, imaging_mono 25x25, tau=1",
                   "packets_per_gpu_per_step": per_gpu,
                   "parallelism": f"packet-sharded x{world}" + (f", one {backend} sum all_reduce per step"
                                                                 if backend else ", single process")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "kernel": "k_trace (dominant: cell-boundary tracing)",
                     "note": "bound: the HBM roofline the contract prices the kernel against (no MFMA work); "
                             "k_trace itself is VALU-issue bound, see limiter (SQ counters of this build)",
                     "alg_bytes_per_packet": round(trace_bpp, 1), "alg_bytes_per_launch": round(per_launch),
                     "avg_launch_ms": round(avg_ms, 4), "launches": t_n,
                     "traffic_source": traffic_src,
                     # what actually limits k_trace (SQ counter passes of this build), if profiled
                     "limiter": limiter,
                     "pipeline": {"kernels": kernels, "ms_per_step": round(k_ms, 3),
                                  "alg_bytes_per_packet": round(b_alg, 1), "achieved_gbs": round(pipeline_gbs, 2),
                                  "step_ms_hip_events": round(float(np.mean(step_ms)), 3)},
                     "events_per_packet": {"crossings": round(C, 3), "scatters": round(S, 4), "peels": round(P, 4)}},
        "cpu_baseline": cpu,
        "engine": engine_info,
        "parity": parity,
        "configs2_32x16x32": cfg2,
        # reference error codes (error.log numbers) logged in the timed steps, with their rate
        "errors": err_rate,
    }
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    if coll:
        tdist.barrier()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

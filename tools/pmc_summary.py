"""Summarise rocprofv3 runs of bench.py into profiles/ (development tool).

Inputs (one bench.py invocation each, same arguments):
  <prof_dir>/trace/run_kernel_stats.csv          rocprofv3 --kernel-trace --stats
  <prof_dir>/pmc_fetch/run_counter_collection.csv rocprofv3 --pmc FETCH_SIZE
  <prof_dir>/pmc_write/run_counter_collection.csv rocprofv3 --pmc WRITE_SIZE

The transport of one bench step is a pipeline of launches (k_trace / k_event / k_emit /
k_rotate per iteration), so bytes are summed over every artes:: kernel of
the profiled run and divided by the packets it transported.

Correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE / WRITE_SIZE are KiB of L2 <-> fabric
requests (HBM and Infinity-Cache hits alike); on gfx950 FETCH_SIZE counts half the bytes
of wide coalesced reads, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  For the
8-byte gathers of this engine the factor 2 is an upper-bound correction.
usage: python tools/pmc_summary.py <prof_dir> <packets_in_profiled_run> <out.json>
The md5 of the profiled libartes_hip.so is recorded: bench.py quotes the traffic only for
the build that was profiled.
"""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict


LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "artes_amd", "lib", "libartes_hip.so")


def rows(path):
    with open(path) as f:
        return [r for r in csv.DictReader(f) if "artes::" in r.get("Kernel_Name", r.get("Name", ""))]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("artes::", "")


def main():
    d, packets, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    stats = rows(os.path.join(d, "trace", "run_kernel_stats.csv"))
    fetch = rows(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = rows(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    per_kernel = defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0})
    for r in fetch:
        per_kernel[short(r["Kernel_Name"])]["fetch_kib"] += float(r["Counter_Value"])
    for r in write:
        per_kernel[short(r["Kernel_Name"])]["write_kib"] += float(r["Counter_Value"])
    f_kb = sum(v["fetch_kib"] for v in per_kernel.values())
    w_kb = sum(v["write_kib"] for v in per_kernel.values())
    hbm = (2.0 * f_kb + w_kb) * 1024.0
    kernels = {}
    for s in stats:
        k = short(s["Name"])
        kernels[k] = {"calls": int(s["Calls"]), "total_ms": float(s["TotalDurationNs"]) / 1e6,
                      "avg_ms": float(s["AverageNs"]) / 1e6, "percent": float(s["Percentage"])}
        if k in per_kernel:
            b = (2.0 * per_kernel[k]["fetch_kib"] + per_kernel[k]["write_kib"]) * 1024.0
            kernels[k]["fabric_bytes_per_packet"] = b / packets
    res = {
        "packets": packets, "fetch_size_kib": f_kb, "write_size_kib": w_kb,
        "hbm_bytes_total": hbm, "hbm_bytes_per_packet": hbm / packets,
        "transport_ms_total": sum(v["total_ms"] for v in kernels.values()),
        "kernels": kernels,
        "lib_md5": hashlib.md5(open(LIB, "rb").read()).hexdigest(),
        "note": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 summed over all artes:: kernels of the profiled "
                "bench run (L2<->fabric requests: HBM and Infinity Cache)",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

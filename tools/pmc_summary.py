"""Summarise rocprofv3 runs of bench.py into profiles/ (development tool).

Reads the kernel-trace stats and the separate FETCH_SIZE / WRITE_SIZE --pmc passes and
writes the transport kernel's per-launch numbers.  Correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half the bytes of a
wide coalesced stream, so HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Float
atomics execute at the memory side and are counted in WRITE_SIZE (64-B requests).
usage: python tools/pmc_summary.py <prof_dir> <packets_per_launch> <out.json>
"""
import csv
import json
import os
import sys


def rows(path, kernel="transport_kernel"):
    with open(path) as f:
        return [r for r in csv.DictReader(f) if kernel in r.get("Kernel_Name", r.get("Name", ""))]


def main():
    d, packets, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    stats = rows(os.path.join(d, "trace", "run_kernel_stats.csv"))
    fetch = rows(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = rows(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    f_kb = sum(float(r["Counter_Value"]) for r in fetch) / max(len(fetch), 1)
    w_kb = sum(float(r["Counter_Value"]) for r in write) / max(len(write), 1)
    hbm = (2.0 * f_kb + w_kb) * 1024.0
    s = stats[0]
    res = {
        "kernel": s["Name"], "calls": int(s["Calls"]), "avg_ms": float(s["AverageNs"]) / 1e6,
        "packets_per_launch": packets, "fetch_size_kib": f_kb, "write_size_kib": w_kb,
        "hbm_bytes_per_launch": hbm, "hbm_bytes_per_packet": hbm / packets,
        "vgpr_count": int(fetch[0]["VGPR_Count"]) if fetch else None,
        "accum_vgpr_count": int(fetch[0]["Accum_VGPR_Count"]) if fetch else None,
        "lds_bytes": int(fetch[0]["LDS_Block_Size"]) if fetch else None,
        "note": "HBM bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE half-count correction); "
                "WRITE_SIZE is dominated by memory-side FP64 detector atomics",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

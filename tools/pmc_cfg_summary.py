"""Per-kernel counter summary of rocprofv3 passes over tools/config_runs.py (development tool).

usage: python tools/pmc_cfg_summary.py <dir with pass subdirs> <config_runs json of the same command> <out.json>

Every subdirectory holds one pass's run_counter_collection.csv (any counter set); counters
are summed per kernel over all dispatches.  Derived (MI355X_MICROARCH.md, HBM / L2 / PMC):
fabric bytes = 2 FETCH_SIZE + WRITE_SIZE KiB (the gfx950 FETCH_SIZE correction), L2 hit rate
TCC_HIT / (TCC_HIT + TCC_MISS), VALU / SALU busy = 4 SQ_INSTS_* / (GRBM_GUI_ACTIVE / 8 x 1024
SIMDs), the wave-cycle split issuing / waiting on memory / issue-stalled, LDS bank-conflict
share of LDS cycles; per scattering event (k_event) and per crossing (k_trace) from the
engine counters of the profiled calls.  A counter collected in more than one pass is
averaged over those passes."""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
# a counter collected in several passes (GRBM_GUI_ACTIVE rides along in three) is averaged
# over them, not summed: each pass profiles the same command
per_pass = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
        per_pass[k][r["Counter_Name"]][f] += float(r["Counter_Value"])
tot = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per_pass.items()}
runs = json.load(open(sys.argv[2]))
calls = [c for key in ("phase", "spectrum") for c in runs.get(key, [])]
packets = sum(c["packets"] for c in calls)
crossings = sum(c["crossings_per_packet"] * c["packets"] for c in calls)
scatters = sum(c["scatters_per_packet"] * c["packets"] for c in calls)
out = {"source": "rocprofv3 --pmc passes of tools/config_runs.py (" + runs.get("config", "") + ")",
       "calls": [c["call"] for c in calls], "packets": packets,
       "crossings_per_packet": round(crossings / packets, 3), "scatters_per_packet": round(scatters / packets, 4),
       "kernels": {}}
for k, c in tot.items():
    if not any(k.startswith(p) for p in ("k_trace", "k_event", "k_emit")):
        continue
    d = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        b = (2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
        d["fabric_bytes_per_packet"] = round(b / packets, 1)
        d["fetch_bytes_per_packet"] = round(2048.0 * c.get("FETCH_SIZE", 0.0) / packets, 1)
        d["write_bytes_per_packet"] = round(1024.0 * c.get("WRITE_SIZE", 0.0) / packets, 1)
    if c.get("TCC_HIT_sum", 0.0) + c.get("TCC_MISS_sum", 0.0) > 0:
        d["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        d["l2_requests_per_packet"] = round((c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) / packets, 2)
    if cyc and "SQ_INSTS_VALU" in c:
        d["valu_busy"] = round(4.0 * c["SQ_INSTS_VALU"] / (cyc * SIMDS), 4)
        d["salu_busy"] = round(4.0 * c.get("SQ_INSTS_SALU", 0.0) / (cyc * SIMDS), 4)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        for name, key in (("wave_cycles_issuing", "SQ_ACTIVE_INST_ANY"), ("wave_cycles_waiting_memory", "SQ_WAIT_ANY"),
                          ("wave_cycles_issue_stalled", "SQ_WAIT_INST_ANY")):
            if key in c:
                d[name] = round(c[key] / wc, 4)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_share"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    unit, n = ("scatter", scatters) if k.startswith("k_event") else (("crossing", crossings) if k.startswith("k_trace") else ("packet", packets))
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS"):
        if name in c:
            d[name.lower().replace("sq_insts_", "") + "_insts_per_" + unit] = round(c[name] / n, 3)
    out["kernels"][k] = d
lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "artes_amd", "lib", "libartes_hip.so")
out["lib_md5"] = hashlib.md5(open(lib, "rb").read()).hexdigest()
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))

"""VALU-issue summary of k_trace / k_event from SQ counter passes (tools/pmc_passes.sh).

usage: python tools/pmc_sq_summary.py <pmc dir> <out.json> [<bench json of the profiled run> <packets>]

Units (MI355X_MICROARCH.md, rocprofv3 PMC section): SQ_INSTS_* count wave-instructions;
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE is
summed over the 8 XCDs.  A wave64 FP64 VALU instruction occupies its SIMD for 4 cycles,
so  VALU busy = 4 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * SIMDs).
With the profiled run's bench line, k_trace's VALU wave-instructions per cell crossing
(lane-level crossings from the engine's counters) are reported too.  The md5 of the
profiled libartes_hip.so is recorded (bench.py quotes the summary only for that build)."""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
tot = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
out = {"source": "rocprofv3 --pmc SQ_* / GRBM_GUI_ACTIVE passes (tools/gpu_round.sh or tools/pmc_passes.sh) of the ray3d transport", "kernels": {}}
for k, c in tot.items():
    if not (k.startswith("k_trace") or k.startswith("k_event") or k.startswith("k_emit")):
        continue
    if "SQ_INSTS_VALU" not in c or "GRBM_GUI_ACTIVE" not in c:
        continue
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    f64 = sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                      "SQ_INSTS_VALU_TRANS_F64"))
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    out["kernels"][k] = {
        "valu_busy": round(4.0 * c["SQ_INSTS_VALU"] / (cycles * SIMDS), 4),
        # SALU wave-instructions take the issuing wave's turn too (4 cycles per SIMD round)
        "salu_busy": round(4.0 * c.get("SQ_INSTS_SALU", 0.0) / (cycles * SIMDS), 4),
        "fp64_arith_share_of_valu": round(f64 / c["SQ_INSTS_VALU"], 4),
        "wave_cycles_issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
        "wave_cycles_waiting_memory": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
        "wave_cycles_issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4),
    }
crossings = None
if len(sys.argv) > 4:
    b = json.load(open(sys.argv[3]))
    crossings = float(b["roofline"]["events_per_packet"]["crossings"]) * float(sys.argv[4])
for k, c in tot.items():
    if k in out["kernels"] and k.startswith("k_trace") and crossings:
        out["kernels"][k]["valu_insts_per_crossing"] = round(c["SQ_INSTS_VALU"] / crossings, 3)
        out["kernels"][k]["salu_insts_per_crossing"] = round(c.get("SQ_INSTS_SALU", 0.0) / crossings, 3)
        out["kernels"][k]["fp64_insts_per_crossing"] = round(
            sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                        "SQ_INSTS_VALU_TRANS_F64")) / crossings, 3)
lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "artes_amd", "lib", "libartes_hip.so")
out["lib_md5"] = hashlib.md5(open(lib, "rb").read()).hexdigest()
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))

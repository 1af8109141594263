"""Summary of tools/pmc_lat.sh's passes: per kernel, average in-flight latency of VMEM / LDS /
SMEM instructions (LEVEL / INSTS, cycles), issue shares per SIMD and lane utilisation."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
grbm = defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
        if not k.startswith("k_"):
            continue
        name, v = r["Counter_Name"], float(r["Counter_Value"])
        if name == "GRBM_GUI_ACTIVE":
            grbm[(k, f)].append(v)
        else:
            tot[k][name] += v
g = defaultdict(float)
for (k, f), vs in grbm.items():
    g[k] += sum(vs) / 3.0   # three passes, the same launches
for k, c in sorted(tot.items()):
    def rat(a, b):
        return c[a] / c[b] if c.get(b) else float("nan")
    simd_cycles = g[k] / 8.0 * 1024   # GRBM_GUI_ACTIVE (summed over the 8 XCDs) -> cycles, x SIMDs
    out = [f"{k}:"]
    out.append(f"vmem lat {c['SQ_INST_LEVEL_VMEM'] / max(c['SQ_INSTS_VMEM_RD'] + c['SQ_INSTS_VMEM_WR'], 1):.0f}")
    out.append(f"lds lat {rat('SQ_INST_LEVEL_LDS', 'SQ_INSTS_LDS'):.0f}")
    out.append(f"smem lat {rat('SQ_INST_LEVEL_SMEM', 'SQ_INSTS_SMEM'):.0f}")
    if simd_cycles:
        for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC"):
            out.append(f"{n.replace('SQ_ACTIVE_INST_', '').lower()} {c[n] * 4 / simd_cycles:.3f}")   # quad-cycles
        out.append(f"valu_busy(insts) {4 * c['SQ_INSTS_VALU'] / simd_cycles:.3f}")
    out.append(f"lanes/valu {rat('SQ_THREAD_CYCLES_VALU', 'SQ_ACTIVE_INST_VALU'):.1f}")
    out.append(f"wait_any {rat('SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):.3f} wait_inst_any {rat('SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES'):.3f} "
               f"wait_inst_lds {rat('SQ_WAIT_INST_LDS', 'SQ_WAVE_CYCLES'):.3f} active_any {rat('SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'):.3f}")
    out.append(f"valu/salu {rat('SQ_INSTS_VALU', 'SQ_INSTS_SALU'):.2f} trans/valu {rat('SQ_INSTS_VALU_TRANS_F64', 'SQ_INSTS_VALU'):.3f} "
               f"branch/valu {rat('SQ_INSTS_BRANCH', 'SQ_INSTS_VALU'):.3f} vmem/valu {(c['SQ_INSTS_VMEM_RD'] + c['SQ_INSTS_VMEM_WR']) / max(c['SQ_INSTS_VALU'], 1):.4f} "
               f"lds/valu {rat('SQ_INSTS_LDS', 'SQ_INSTS_VALU'):.3f} smem/valu {rat('SQ_INSTS_SMEM', 'SQ_INSTS_VALU'):.3f} bankconf/lds {rat('SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_LDS'):.2f}")
    print(" ".join(out))

#!/bin/bash
# k_event LDS-layout A/B of the cumulative sampling tables on the configs[3] cloudy calls
# (development tool): per build (tags as tools/ab_run.sh) the cloudy call
# timings (tools/ab_cfg.sh: 2 phase angles + 2 wavelengths at 1e8) and one counter pass of the
# same calls for k_event's LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
# usage (via gpurun): bash tools/gpu_lds_layout_ab.sh <out> <tag> [<tag> ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 bash tools/ab_cfg.sh $O/cfg "$@" "$@" > $O/cfg.txt 2>&1 || { tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt
for L in "$@"; do
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_$L -o run -- python3 tools/config_runs.py $O/pmcrun_$L --which 3 --packets 1e8 --phases 2 --lambdas 2 \
    > $O/pmc_$L.log 2>&1 || { echo "pmc $L failed"; tail -5 $O/pmc_$L.log; exit 1; }
  python3 - $O/pmc_$L/run_counter_collection.csv $L <<'PY'
import csv, sys
from collections import defaultdict
t = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in t.items():
    if k.startswith("k_event"):
        share = c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
        print(f"[{sys.argv[2]}] {k}: lds_bank_conflict_share {share:.4f}  SQ_LDS_BANK_CONFLICT={c['SQ_LDS_BANK_CONFLICT']:.4g} "
              f"SQ_LDS_IDX_ACTIVE={c['SQ_LDS_IDX_ACTIVE']:.4g} SQ_INSTS_LDS={c['SQ_INSTS_LDS']:.4g} SQ_WAVE_CYCLES={c['SQ_WAVE_CYCLES']:.4g}")
PY
done

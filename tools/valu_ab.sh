#!/bin/bash
# VALU / SALU wave-instructions of k_trace per cell crossing for several library builds
# (one rocprofv3 --pmc pass each over tools/prof_one.py; development tool).
# usage (via gpurun): bash tools/valu_ab.sh <tag> <config> <packets> <lib> [<lib> ...]
set -o pipefail
TAG=$1; CFG=$2; N=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for LIB in "$@"; do
  i=$((i+1))
  ARTES_LIB_PATH=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/v$i -o run -- python3 tools/prof_one.py $CFG $N > $OUT/v$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/v$i.log; exit 1; }
  echo "== $LIB"; grep -v amdgpu $OUT/v$i.log
  python3 - $OUT/v$i/run_counter_collection.csv <<'PY'
import csv, sys
from collections import defaultdict
t = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in t.items():
    if k.startswith("k_"):
        print(f"  {k}: " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
PY
done

#!/bin/bash
# VALU / SALU wave-instructions of k_trace for several environment settings of one library
# (one rocprofv3 --pmc pass each over tools/prof_one.py; development tool).
# usage (via gpurun): bash tools/valu_env.sh <tag> <config> <packets> "<ENV=V ...>" ["<ENV=V ...>" ...]
set -o pipefail
TAG=$1; CFG=$2; N=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "$@"; do
  i=$((i+1))
  ( export $SET; timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/e$i -o run -- python3 tools/prof_one.py $CFG $N > $OUT/e$i.log 2>&1 ) || { echo "pass $i failed"; tail -5 $OUT/e$i.log; exit 1; }
  echo "== $SET"; grep "pkt/s" $OUT/e$i.log
  python3 - $OUT/e$i/run_counter_collection.csv <<'PY'
import csv, sys
from collections import defaultdict
t = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in t.items():
    if k.startswith("k_trace"):
        print(f"  {k}: " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
PY
done

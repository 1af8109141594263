#!/bin/bash
# Separate rocprofv3 --pmc passes over one short engine run (development tool).
# usage (via gpurun): bash tools/pmc_passes.sh <tag> <config> <packets> "<pass1 counters>" ["<pass2 counters>" ...]
set -o pipefail
TAG=$1; CFG=$2; N=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/prof_one.py $CFG $N > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt

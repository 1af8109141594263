#!/bin/bash
set -o pipefail
O=gpurun_out/r05ta; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt || true
i=0
for set in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum" "TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum"; do
  i=$((i+1)); ok=1
  for c in $set; do b=${c%_sum}; grep -qx "$b" $O/names.txt || [ "$c" = GRBM_GUI_ACTIVE ] || ok=0; done
  [ $ok = 1 ] || { echo "skip $set"; continue; }
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/prof_one.py ray3d 1e8 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
  echo "== $set"; python3 tools/pmc_kernels.py $O/p$i/run_counter_collection.csv
done

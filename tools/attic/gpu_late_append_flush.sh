#!/bin/bash
# late append with the off-critical-path queue flush: knob on/off on every workload
set -o pipefail
O=gpurun_out/late_flush; mkdir -p $O
timeout -k 10 300 python tools/quick_perf.py 3e8 "ARTES_LATE_APPEND=0" "ARTES_LATE_APPEND=1" > $O/qp.txt 2>&1 || { echo qp failed; tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu $O/qp.txt
timeout -k 10 400 bash tools/cfg_env_sweep.sh $O/cfg "ARTES_LATE_APPEND=0" "ARTES_LATE_APPEND=1" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt

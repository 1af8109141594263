#!/bin/bash
set -o pipefail
O=gpurun_out/s4; mkdir -p $O
LS_WORKLOAD=cloudy ARTES_LIB_PATH=$PWD/artes_amd/lib/libartes_hip_lanes.so timeout -k 10 200 python tools/lane_stats.py 1e8 > $O/lanes_cloudy.txt 2>&1 || { tail -5 $O/lanes_cloudy.txt; exit 1; }
grep -v amdgpu.ids $O/lanes_cloudy.txt
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_REFILL=8" "ARTES_REFILL=24" "ARTES_REFILL=32" "ARTES_HBATCH=2" "ARTES_HBATCH=10" "ARTES_STATIC=32" "ARTES_STATIC=64" "ARTES_EMIT_FIRST=1" "ARTES_BACKWARD=0" "ARTES_EVENT_BLOCK=256" "ARTES_PIX1=0"

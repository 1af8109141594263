#!/bin/bash
# Lane accounting (-DARTES_DEBUG_LANES) and region timing (-DARTES_DEBUG_TIMING) of k_trace on
# ray3d and the cloudy phase call (development tool).
# usage (via gpurun): bash tools/gpu_lanes_regions.sh <out> [packets]
export ARTES_DEV_LIB=1   # (development builds load only with this opt-in: artes_amd/engine.py)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
N=${2:-1e8}
for W in ray3d cloudy; do
  LS_WORKLOAD=$W ARTES_LIB_PATH=artes_amd/lib/libartes_hip_lanes.so timeout -k 10 200 python tools/lane_stats.py $N > $O/lanes_$W.txt 2>&1 || { tail -5 $O/lanes_$W.txt; exit 1; }
  grep -v amdgpu $O/lanes_$W.txt
done
bash tools/gpu_time_regions.sh $1/tr $N

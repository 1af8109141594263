#!/bin/bash
# k_trace region timing (the -DARTES_DEBUG_TIMING build) on ray3d and the cloudy calls.
# usage (via gpurun): bash tools/gpu_time_regions.sh <out> [packets] [ENV=V,...]...
export ARTES_DEV_LIB=1   # (development builds load only with this opt-in: artes_amd/engine.py)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
N=${1:-1e8}; shift
export ARTES_LIB_PATH=artes_amd/lib/libartes_hip_timing.so
timeout -k 10 200 python tools/time_regions.py $N "$@" > $O/ray3d.txt 2>&1 || { tail -5 $O/ray3d.txt; exit 1; }
cat $O/ray3d.txt
LS_WORKLOAD=cloudy timeout -k 10 200 python tools/time_regions.py $N "$@" > $O/cloudy.txt 2>&1 || { tail -5 $O/cloudy.txt; exit 1; }
cat $O/cloudy.txt

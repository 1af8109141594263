#!/bin/bash
# Round-6 A/B session (development tool): trajectory agreement and ray3d / hg / iso timing of
# several engine builds (tags as tools/ab_run.sh), then the early-exit knob sweep on the last one.
# usage (via gpurun): bash tools/gpu_ab_r06.sh <out> <packets> <tag> [<tag> ...]
set -o pipefail
O=gpurun_out/$1; N=$2; shift 2; mkdir -p $O
LAST=""
for L in "$@"; do
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  echo "== $L"
  ARTES_LIB_PATH=$P timeout -k 10 300 python tools/quick_perf.py $N "" > $O/$L.txt 2>&1 || { echo "run $L failed"; tail -5 $O/$L.txt; exit 1; }
  grep -v amdgpu.ids $O/$L.txt
  LAST=$P
done
[ -z "$EARLY" ] && exit 0   # (the early-exit knob was not kept: set EARLY=1 with a build that has it)
echo "== early sweep on $LAST"
QP_CHECK=0 ARTES_LIB_PATH=$LAST timeout -k 10 400 python tools/quick_perf.py $N "" ARTES_EARLY=16 ARTES_EARLY=24 ARTES_EARLY=32 ARTES_EARLY=40 > $O/early.txt 2>&1 || { echo "sweep failed"; tail -5 $O/early.txt; exit 1; }
grep -v amdgpu.ids $O/early.txt

#!/bin/bash
# Time several engine builds back to back on one box (development tool).
# usage (via gpurun): bash tools/ab_run.sh <packets> <tag> [<tag> ...]   (tag "cur" = artes_amd/lib/libartes_hip.so)
N=$1; shift
export QP_CHECK=${QP_CHECK:-0}
for L in "$@"; do
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  echo "== $L"
  ARTES_LIB_PATH=$P timeout -k 10 200 python tools/quick_perf.py $N "" > gpurun_out/ab_$L.log 2>&1 || { echo "run $L failed"; tail -5 gpurun_out/ab_$L.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$L.log
done

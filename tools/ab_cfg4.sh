#!/bin/bash
# configs[4] thermal spectrum (100 wavelengths at 1e8) for several engine builds (development tool)
# usage (via gpurun): bash tools/ab_cfg4.sh <out dir> <tag> [<tag> ...]   (tag "cur" = artes_amd/lib/libartes_hip.so)
set -o pipefail
O=$1; shift; mkdir -p $O
for L in "$@"; do
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python tools/config_runs.py $O/$L --which 4 --packets 1e8 > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  echo "[$L]: $(tail -1 $O/$L.log)"
done

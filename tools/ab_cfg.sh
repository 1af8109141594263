#!/bin/bash
# configs[3] cloudy calls (2 phase angles + 2 wavelengths at 1e8) for several engine builds,
# back to back on one box (development tool).
# usage (via gpurun): bash tools/ab_cfg.sh <out dir> <tag> [<tag> ...]   (tag "cur" = artes_amd/lib/libartes_hip.so)
set -o pipefail
O=$1; shift; mkdir -p $O
for L in "$@"; do
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 200 python tools/config_runs.py $O/$L --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  echo "[$L]: $(grep '"what"' $O/$L.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
  grep '"call"' $O/$L.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d["kernel_ms"]; print("   ", d["call"], d["mpackets_per_s"], " ".join(f"{a} {b:.0f}" for a,b in k.items()))'
done

#!/bin/bash
# configs[3] cloudy calls (2 phase angles + 2 wavelengths at 1e8) for several library tags
# and launch-knob variants (development tool).
# usage (via gpurun): bash tools/gpu_cfg_variants.sh <out> <tag>:<ENV=V,ENV=V|-> [...]   (tag "cur" = libartes_hip.so)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for tv in "$@"; do
  L=${tv%%:*}; v=${tv#*:}; [ "$v" = "-" ] && v=""
  if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  tag=$(echo "$tv" | tr ',=:' '___')
  ( if [ -n "$v" ]; then export $(echo "$v" | tr ',' ' '); fi
    ARTES_LIB_PATH=$P timeout -k 10 200 python tools/config_runs.py $O/$tag --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/$tag.log 2>&1 ) || { tail -5 $O/$tag.log; exit 1; }
  echo "[$tv]: $(grep '"what"' $O/$tag.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
  grep '"call"' $O/$tag.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d["kernel_ms"]; print("   ", d["call"], d["mpackets_per_s"], " ".join(f"{a} {b:.0f}" for a,b in k.items()))'
done

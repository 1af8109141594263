#!/bin/bash
# configs[3] cloudy calls (2 phase angles + 2 wavelengths at 1e8) of the current library for
# each tuning variant "ARTES_KEY=V[,...]" ("" = defaults), applied through artes_set_tuning
# (tools/_tuning.py); development tool.
# usage (via gpurun): bash tools/gpu_cfg_knobs_r05.sh <out> <variant> [<variant> ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for v in "$@"; do
  tag=$(echo "$v" | tr ',=' '__'); [ -z "$tag" ] && tag=default
  ( if [ -n "$v" ]; then export $(echo "$v" | tr ',' ' '); fi
    timeout -k 10 200 python tools/config_runs.py $O/cfg_$tag --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/cfg_$tag.log 2>&1 ) || { tail -5 $O/cfg_$tag.log; exit 1; }
  echo "[cloudy $v]: $(grep '"what"' $O/cfg_$tag.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
done

#!/bin/bash
# launch-knob sweep on the configs[3] cloudy calls (2 phase angles + 2 wavelengths at 1e8)
# usage: bash tools/cfg_env_sweep.sh <out dir> "ENV=V ENV2=V2" ...   ("" = defaults)
set -o pipefail
O=$1; shift; mkdir -p $O
i=0
for VAR in "$@"; do
  i=$((i+1))
  env $VAR timeout -k 10 200 python tools/config_runs.py $O/v$i --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/v$i.log 2>&1 || { tail -5 $O/v$i.log; exit 1; }
  echo "[$VAR]: $(grep '"what"' $O/v$i.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
done

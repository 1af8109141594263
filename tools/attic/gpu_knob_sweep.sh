#!/bin/bash
# Launch-knob sweep of the current library (development tool): ray3d / hg / iso at 3e8
# (production settings: packet moments off) and the configs[3] cloudy calls (2 phase angles
# + 2 wavelengths at 1e8), one run per variant "ENV=V[,ENV=V]" ("" = defaults), plus the
# base library for reference.
# usage (via gpurun): bash tools/gpu_knob_sweep.sh <out> <variant> [<variant> ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 150 python tools/quick_perf.py 1e6 > $O/traj.log 2>&1 || { echo traj failed; tail -20 $O/traj.log; exit 1; }
grep agreement $O/traj.log
if [ -f artes_amd/lib/libartes_hip_base.so ]; then
  QP_CHECK=0 QP_MOMENTS=0 ARTES_LIB_PATH=artes_amd/lib/libartes_hip_base.so timeout -k 10 300 python tools/quick_perf.py 3e8 "" > $O/base.txt 2>&1 || { echo base failed; tail -5 $O/base.txt; exit 1; }
  echo "== base"; grep -v amdgpu $O/base.txt
fi
QP_CHECK=0 QP_MOMENTS=0 timeout -k 10 600 python tools/quick_perf.py 3e8 "$@" > $O/knobs.txt 2>&1 || { echo knobs failed; tail -5 $O/knobs.txt; exit 1; }
echo "== cur"; grep -v amdgpu $O/knobs.txt
for v in "$@"; do
  tag=$(echo "$v" | tr ',=' '__'); [ -z "$tag" ] && tag=default
  if [ -n "$v" ]; then export $(echo "$v" | tr ',' ' '); fi
  timeout -k 10 200 python tools/config_runs.py $O/cfg_$tag --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/cfg_$tag.log 2>&1 || { tail -5 $O/cfg_$tag.log; exit 1; }
  if [ -n "$v" ]; then unset $(echo "$v" | tr ',' ' ' | sed 's/=[^ ]*//g'); fi
  echo "[cloudy $v]: $(grep '"what"' $O/cfg_$tag.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
  grep '"call"' $O/cfg_$tag.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d["kernel_ms"]; print("   ", d["call"], d["mpackets_per_s"], " ".join(f"{a} {b:.0f}" for a,b in k.items()))'
done
if [ -f artes_amd/lib/libartes_hip_base.so ]; then
  ARTES_LIB_PATH=artes_amd/lib/libartes_hip_base.so timeout -k 10 200 python tools/config_runs.py $O/cfg_base --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/cfg_base.log 2>&1 || { tail -5 $O/cfg_base.log; exit 1; }
  echo "[cloudy base]: $(grep '"what"' $O/cfg_base.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phase_summary"]["mpackets_per_s"], d["spectrum_summary"]["mpackets_per_s"])')"
fi

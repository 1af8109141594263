#!/bin/bash
# trace-list order and static share on the current build (3e8 ray3d / hg / iso; cloudy calls at 1e8)
set -o pipefail
O=gpurun_out/order; mkdir -p $O
QP_CHECK=0 timeout -k 10 600 python tools/quick_perf.py 3e8 "" "ARTES_EMIT_FIRST=1" "ARTES_EMIT_FIRST=0" "ARTES_STATIC=40" "ARTES_STATIC=56" > $O/qp.txt 2>&1 || { echo qp failed; tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu $O/qp.txt
timeout -k 10 600 bash tools/cfg_env_sweep.sh $O/cfg "" "ARTES_EMIT_FIRST=1" "ARTES_STATIC=56" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt

#!/bin/bash
set -o pipefail
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_perf.py 3e8 "" "ARTES_KLDS=0" > $O/qp.txt 2>&1 || { tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu.ids $O/qp.txt
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_KLDS=0" "ARTES_REFILL=32 ARTES_EMIT_FIRST=1"

#!/bin/bash
# the oblate case under the checked build with the doubled trace lists, then the GPU suite
set -o pipefail
O=gpurun_out/s7; mkdir -p $O
D=$PWD/artes_amd/lib/libartes_hip_debug.so
ARTES_LIB_PATH=$D timeout -k 10 120 python tools/oblate_probe.py > $O/oblate_debug.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/oblate_debug.txt; [ $rc -eq 0 ] || exit $rc
grep -q '"ok": true' $O/oblate_debug.txt || { echo "checked build still fails"; exit 3; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_perf.py 3e8 "" "ARTES_KLDS=0" > $O/qp.txt 2>&1 || { tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu.ids $O/qp.txt
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_KLDS=0" "ARTES_REFILL=32 ARTES_EMIT_FIRST=1"

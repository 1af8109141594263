#!/bin/bash
set -o pipefail
O=gpurun_out/s8; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_EVENT_LDSC=0" "ARTES_REFILL=32 ARTES_EMIT_FIRST=1" "ARTES_REFILL=32"
ARTES_VERBOSE=1 timeout -k 10 200 python tools/config_runs.py $O/one --which 3 --packets 1e7 --phases 1 --lambdas 1 2>&1 | grep "event engine" | head -3

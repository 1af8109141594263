#!/bin/bash
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cloudy.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/config_runs.py $O/cfg --which 3 --packets 1e9 --phases 19 --lambdas 13 > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; exit 1; }
tail -1 $O/cfg.log

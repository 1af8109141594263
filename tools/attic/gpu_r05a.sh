#!/bin/bash
# Round 5, first session: the GPU suite on the tuning-API build, then the baseline timings
# (ray3d / hg / iso at 3e8 with the production settings, the cloudy configs[3] calls).
# usage (via gpurun): bash tools/gpu_r05a.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
QP_CHECK=0 QP_MOMENTS=0 timeout -k 10 300 python tools/quick_perf.py 3e8 > $O/qp.txt 2>&1 || { echo qp failed; tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu $O/qp.txt
timeout -k 10 300 python tools/config_runs.py $O/cfg --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; exit 1; }
grep '"what"' $O/cfg.log | tail -1

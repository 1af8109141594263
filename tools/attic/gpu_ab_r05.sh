#!/bin/bash
# A/B session (development tool): trajectory agreement of the current library, ray3d / hg /
# iso timing (3e8, production settings) and the cloudy configs[3] calls of the current library
# against libartes_hip_base.so, k_trace VALU / SALU per crossing of both, then the GPU suite.
# usage (via gpurun): bash tools/gpu_ab_r05.sh <out> [nosuite]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 150 python tools/quick_perf.py 1e6 > $O/traj.log 2>&1 || { echo traj failed; tail -20 $O/traj.log; exit 1; }
grep agreement $O/traj.log
export QP_MOMENTS=0
timeout -k 10 600 bash tools/ab_run.sh 3e8 base cur base cur > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 600 bash tools/ab_cfg.sh $O/cfg base cur > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt
timeout -k 10 300 bash tools/valu_ab.sh $1/valu ray3d 1e8 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $O/valu.txt 2>&1 || { echo "valu pass failed"; tail -5 $O/valu.txt; exit 1; }
cat $O/valu.txt
if [ "$2" != nosuite ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi

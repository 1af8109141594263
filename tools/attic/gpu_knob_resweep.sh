#!/bin/bash
# knob re-sweep on the current build (after the late appends): refill threshold, interaction
# batch, pool size on ray3d / hg / iso (3e8) and the cloudy calls (1e8)
set -o pipefail
O=gpurun_out/knobs; mkdir -p $O
timeout -k 10 150 python tools/quick_perf.py 1e6 > $O/traj.log 2>&1 || { echo traj failed; tail -20 $O/traj.log; exit 1; }
grep agreement $O/traj.log
QP_CHECK=0 timeout -k 10 600 python tools/quick_perf.py 3e8 "" "ARTES_REFILL=12" "ARTES_REFILL=20" "ARTES_REFILL=24" "ARTES_HBATCH=4" "ARTES_HBATCH=8" "ARTES_POOL=50331648" > $O/qp.txt 2>&1 || { echo qp failed; tail -5 $O/qp.txt; exit 1; }
grep -v amdgpu $O/qp.txt
timeout -k 10 600 bash tools/cfg_env_sweep.sh $O/cfg "" "ARTES_REFILL=24" "ARTES_REFILL=40" "ARTES_HBATCH=4" "ARTES_HBATCH=8" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt

#!/bin/bash
# A/B of the current library against libartes_hip_base.so (development tool): trajectory
# agreement, ray3d/hg/iso timing, k_trace VALU/SALU per crossing, then the GPU suite.
# usage (via gpurun): bash tools/gpu_ab_valu.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 150 python tools/quick_perf.py 1e6 > $O/traj.log 2>&1 || { echo traj failed; tail -20 $O/traj.log; exit 1; }
grep agreement $O/traj.log
timeout -k 10 600 bash tools/ab_run.sh 3e8 base cur base cur > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 bash tools/valu_ab.sh $1/valu ray3d 1e8 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $O/valu.txt 2>&1 || { echo "valu pass failed"; tail -5 $O/valu.txt; exit 1; }
cat $O/valu.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log

#!/bin/bash
# One GPU session for a k_trace change (development tool): trajectory agreement of the
# current library on ray3d / hg / iso, the GPU test suite, SQ_INSTS_VALU of k_trace for
# the baseline (libartes_hip_base.so, tools/ab_build.sh) and the current library, and
# their throughput back to back.
# usage (via gpurun): bash tools/ab_gpu.sh <tag> [packets]
set -o pipefail
TAG=$1; N=${2:-3e8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 python tools/quick_perf.py 1e6 > $OUT/traj.log 2>&1 || { echo "trajectory check failed"; tail -5 $OUT/traj.log; exit 1; }
grep agreement $OUT/traj.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 bash tools/valu_ab.sh $TAG ray3d 1e8 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $OUT/valu.txt 2>&1 || { echo "valu pass failed"; tail -5 $OUT/valu.txt; exit 1; }
grep "==\|k_trace\|pkt/s" $OUT/valu.txt
QP_CHECK=0 timeout -k 10 400 bash tools/ab_run.sh $N base cur base cur > $OUT/ab.txt 2>&1 || { echo "timing failed"; tail -5 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt

#!/bin/bash
# The GPU suite on the current build, then it against libartes_hip_base.so: ray3d / hg / iso at
# 3e8 (production settings) and the cloudy calls.   usage (via gpurun): bash tools/gpu_check_ab.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
QP_MOMENTS=0 timeout -k 10 600 bash tools/ab_run.sh 3e8 base cur base cur > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
bash tools/gpu_cfg_variants.sh $1c base:- cur:-

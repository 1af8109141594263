#!/bin/bash
# Launch-schedule sweep of the current library through artes_set_tuning (development tool):
# ray3d / hg / iso at 3e8 (production settings) for each variant "ARTES_KEY=V[,...]", twice.
# usage (via gpurun): bash tools/gpu_knobs_r05.sh <out> <variant> [<variant> ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
QP_CHECK=0 QP_MOMENTS=0 timeout -k 10 900 python tools/quick_perf.py 3e8 "$@" "$@" > $O/knobs.txt 2>&1 || { echo knobs failed; tail -5 $O/knobs.txt; exit 1; }
grep -v amdgpu $O/knobs.txt

#!/bin/bash
# ARTES_NREP A/B (development tool): the trajectory check of each rep build, ray3d / hg / iso at
# 3e8 (production settings) and the cloudy calls, for the library tags given (cur = NREP of the
# shipping build).   usage (via gpurun): bash tools/gpu_rep_ab.sh <out> <tag> [<tag> ...]
set -o pipefail
O=$1; shift
mkdir -p gpurun_out/$O
for t in "$@"; do
  [ "$t" = cur ] && continue
  ARTES_LIB_PATH=artes_amd/lib/libartes_hip_$t.so timeout -k 10 150 python tools/quick_perf.py 1e6 > gpurun_out/$O/traj_$t.log 2>&1 || exit 1
  echo "$t: $(grep agreement gpurun_out/$O/traj_$t.log | tr '\n' ' ')"
done
QP_MOMENTS=0 timeout -k 10 700 bash tools/ab_run.sh 3e8 "$@" > gpurun_out/$O/ab.txt 2>&1 || exit 1
cat gpurun_out/$O/ab.txt
bash tools/gpu_cfg_variants.sh ${O}c $(for t in "$@"; do echo -n "$t:- "; done)

#!/bin/bash
# A/B of engine builds (development tool): ray3d / hg / iso at 3e8 in the production
# configuration (packet moments off), then the configs[3] cloudy calls (2 phase angles + 2
# wavelengths at 1e8), for every tag (tags as tools/ab_run.sh), twice over.
# usage (via gpurun): bash tools/gpu_ab_knobs.sh <out> <tag> [<tag> ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
QP_MOMENTS=0 timeout -k 10 700 bash tools/ab_run.sh 3e8 "$@" "$@" > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 700 bash tools/ab_cfg.sh $O/cfg "$@" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt

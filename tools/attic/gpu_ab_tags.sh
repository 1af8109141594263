#!/bin/bash
# A/B of several engine builds (development tool): ray3d / hg / iso at 3e8 (production
# settings) and the cloudy configs[3] calls, each build back to back on one box, twice.
# usage (via gpurun): bash tools/gpu_ab_tags.sh <out> <tag> [<tag> ...]   (tag "cur" = libartes_hip.so)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export QP_MOMENTS=0
timeout -k 10 600 bash tools/ab_run.sh 3e8 "$@" "$@" > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 600 bash tools/ab_cfg.sh $O/cfg "$@" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt

#!/bin/bash
# One A/B session (development tool): trajectory agreement of the current library, timing of
# the given builds on ray3d / hg / iso and the cloudy configs[3] calls, then the GPU suite.
# usage (via gpurun): bash tools/gpu_ab3.sh <out> <tag> [<tag> ...]   (tags as tools/ab_run.sh)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 150 python tools/quick_perf.py 1e6 > $O/traj.log 2>&1 || { echo traj failed; tail -20 $O/traj.log; exit 1; }
grep agreement $O/traj.log
timeout -k 10 600 bash tools/ab_run.sh 3e8 "$@" "$@" > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 600 bash tools/ab_cfg.sh $O/cfg "$@" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log

#!/bin/bash
# lookahead refills (libartes_hip_la.so, -DARTES_LOOKAHEAD) against the default build across
# refill thresholds: cloudy configs[3] calls at 1e8 and ray3d / hg / iso at 3e8
set -o pipefail
O=gpurun_out/la_refill; mkdir -p $O
LA=artes_amd/lib/libartes_hip_la.so
timeout -k 10 900 bash tools/cfg_env_sweep.sh $O/cfg "ARTES_REFILL=32" "ARTES_LIB_PATH=$LA ARTES_REFILL=32" "ARTES_REFILL=16" "ARTES_LIB_PATH=$LA ARTES_REFILL=16" "ARTES_LIB_PATH=$LA ARTES_REFILL=24" > $O/cfg.txt 2>&1 || { echo cfg failed; tail -5 $O/cfg.txt; exit 1; }
cat $O/cfg.txt
QP_CHECK=0 timeout -k 10 600 bash tools/ab_run.sh 3e8 cur la > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt

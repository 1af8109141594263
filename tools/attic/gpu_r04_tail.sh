#!/bin/bash
# smoke() and the k_trace region timing on the final round-4 build, then cloudy launch-knob
# and theta-two-face (libartes_hip_th2.so) variants (development session).
set -o pipefail
mkdir -p gpurun_out/r04t
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04t/smoke.log 2>&1 || { tail -20 gpurun_out/r04t/smoke.log; exit 1; }
tail -3 gpurun_out/r04t/smoke.log
bash tools/gpu_time_regions.sh r04t/tr 1e8 || exit 1
ARTES_LIB_PATH=artes_amd/lib/libartes_hip_th2.so timeout -k 10 150 python tools/quick_perf.py 1e6 > gpurun_out/r04t/th2_traj.log 2>&1 || { tail -5 gpurun_out/r04t/th2_traj.log; exit 1; }
grep agreement gpurun_out/r04t/th2_traj.log
bash tools/gpu_cfg_variants.sh r04t/cv cur:- cur:ARTES_REFILL=20 cur:ARTES_GBATCH=8 cur:ARTES_REFILL=20,ARTES_GBATCH=8 th2:- cur:- cur:ARTES_REFILL=20,ARTES_GBATCH=8 th2:-

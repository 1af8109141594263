#!/bin/bash
# A/B of k_event builds (development tool): ray3d / hg / iso timing in the production
# configuration (packet moments off, as bench.py and the CLI run), and one SQ pass per
# library over the ray3d and cloudy commands (VALU / LDS / VMEM instructions, wave cycles).
# usage (via gpurun): bash tools/gpu_ab_ev.sh <out> <tag> [<tag> ...]   (tags as tools/ab_run.sh)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
QP_MOMENTS=0 timeout -k 10 600 bash tools/ab_run.sh 3e8 "$@" "$@" > $O/ab.txt 2>&1 || { echo ab failed; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
for cfg in ray3d cloudy; do
  for L in "$@"; do
    if [ "$L" = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
    ARTES_LIB_PATH=$P timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/sq_${cfg}_$L -o run -- python3 tools/prof_one.py $cfg 1e8 > $O/sq_${cfg}_$L.log 2>&1 || { echo "sq $cfg $L failed"; tail -5 $O/sq_${cfg}_$L.log; exit 1; }
    echo "== $cfg $L: $(grep -v amdgpu $O/sq_${cfg}_$L.log | tail -1)"
    python3 tools/pmc_kernels.py $O/sq_${cfg}_$L/run_counter_collection.csv
  done
done

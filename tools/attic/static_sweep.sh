#!/bin/bash
# Sweep the trace-list distribution knobs of k_trace (development tool): the statically
# dealt share of the list (ARTES_STATIC, in 1/64) and the idle-lane refill threshold
# (ARTES_REFILL), on ray3d / hg / iso.
# usage (via gpurun): bash tools/static_sweep.sh [packets]
N=${1:-3e8}
V=""
for sr in 32,24 40,20 48,20 48,24 56,20 56,24 64,24 48,32 56,28 56,32 64,32; do
  V="$V ARTES_STATIC=${sr%,*},ARTES_REFILL=${sr#*,}"
done
mkdir -p gpurun_out
QP_MOMENTS=0 QP_CHECK=0 timeout -k 10 500 python -u tools/quick_perf.py $N '' $V > gpurun_out/static_sweep.log 2>&1
grep pkt gpurun_out/static_sweep.log

#!/bin/bash
mkdir -p gpurun_out/pool
export QP_CHECK=0 ARTES_VERBOSE=1
for P in 4194304 8388608 16777216 33554432; do
  echo "== pool $P"
  ARTES_POOL=$P timeout -k 10 200 python tools/quick_perf.py 4e8 "" > gpurun_out/pool/p$P.log 2>&1 || { echo "failed $P"; tail -5 gpurun_out/pool/p$P.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/pool/p$P.log | grep -v "1e+05\|100000 " | tail -8
done

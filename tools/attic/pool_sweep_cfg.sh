#!/bin/bash
# pool-size sweep on the configs[3] cloudy calls (2 phase angles + 2 wavelengths at 1e8) and
# the bench-shaped ray3d transport; usage: bash tools/pool_sweep_cfg.sh <out dir> <pool sizes...>
set -o pipefail
O=$1; shift; mkdir -p $O
for P in "$@"; do
  ARTES_POOL=$P timeout -k 10 200 python tools/config_runs.py $O/p$P --which 3 --packets 1e8 --phases 2 --lambdas 2 > $O/cfg_p$P.log 2>&1 || { tail -5 $O/cfg_p$P.log; exit 1; }
  echo "pool $P: $(grep '"what"' $O/cfg_p$P.log | tail -1)"
  ARTES_POOL=$P QP_CHECK=0 timeout -k 10 200 python tools/quick_perf.py 3e8 > $O/qp_p$P.log 2>&1 || { tail -5 $O/qp_p$P.log; exit 1; }
  grep -v amdgpu.ids $O/qp_p$P.log | head -1
done

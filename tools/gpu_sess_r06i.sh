#!/bin/bash
# Round-6 session i (development tool): k_trace steps per iteration on fine grids (ARTES_FINE_NREP
# builds 6 / 10 / 12 against the shipping 8): ray3d / hg / iso (tools/quick_perf.py) and the bench grid.
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 bash tools/gpu_ab_r06.sh r06j 3e8 cur rep9 rep10 rep11 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
for L in cur rep9 rep10 rep11 cur rep9 rep10 rep11; do
  if [ $L = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variants > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done

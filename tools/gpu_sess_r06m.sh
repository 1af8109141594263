#!/bin/bash
# Round-6 session m (development tool): the radial-form runaway test once per iteration and the
# unconditional face update, against the profiled round-6 build (r06a): timing, bench grid, VALU.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 900 bash tools/gpu_ab_r06.sh r06m 3e8 r06a cur > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
for L in r06a cur r06a cur; do
  if [ $L = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variants > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done
timeout -k 10 300 bash tools/valu_ab.sh r06m/valu ray3d 1e8 artes_amd/lib/libartes_hip_r06a.so artes_amd/lib/libartes_hip.so > $O/valu.txt 2>&1 || { tail -5 $O/valu.txt; exit 1; }
grep "k_trace" $O/valu.txt

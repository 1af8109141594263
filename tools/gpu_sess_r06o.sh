#!/bin/bash
# Round-6 session o (development tool): k_trace slot variants against the profiled build (cur):
# vB the slot's still-stepping lanes as a lane mask, vC vB + the radial pending bit as a lane mask,
# vE the radial pending bit alone.  Trajectory agreement + ray3d / hg / iso timing, bench grid, VALU.
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
LIBS="${LIBS:-cur vB vC vE}"
timeout -k 10 900 bash tools/gpu_ab_r06.sh r06o 3e8 $LIBS > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
for L in $LIBS cur; do
  if [ $L = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variants > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done
PL=""; for L in $LIBS; do if [ $L = cur ]; then PL="$PL artes_amd/lib/libartes_hip.so"; else PL="$PL artes_amd/lib/libartes_hip_$L.so"; fi; done
timeout -k 10 400 bash tools/valu_ab.sh r06o/valu ray3d 1e8 $PL > $O/valu.txt 2>&1 || { tail -5 $O/valu.txt; exit 1; }
grep "k_trace\|==" $O/valu.txt

#!/bin/bash
# Round-6 session q (development tool): engine builds against the profiled one (cur) -- trajectory
# agreement, ray3d / hg / iso timing and the bench command, twice each in alternation.
# usage (via gpurun): LIBS="cur em4 em5" bash tools/gpu_sess_r06q.sh <out>
set -o pipefail
T=${1:-r06q}; O=gpurun_out/$T; mkdir -p $O
LIBS="${LIBS:-cur em4 em5}"
timeout -k 10 900 bash tools/gpu_ab_r06.sh $T 3e8 $LIBS > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
for L in $LIBS $LIBS; do
  if [ $L = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variants > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done

#!/bin/bash
# Round-6 session s (development tool): the current build (cur) against the previous one (r06r):
# trajectory agreement, ray3d / hg / iso timing, the bench command twice each, VALU per crossing,
# then the GPU test suite on the current build (NOTEST=1: not).
# usage (via gpurun): LIBS="r06r cur" bash tools/gpu_sess_r06s.sh <out>
set -o pipefail
T=${1:-r06s}; O=gpurun_out/$T; mkdir -p $O
LIBS="${LIBS:-r06r cur}"
timeout -k 10 600 bash tools/gpu_ab_r06.sh $T 3e8 $LIBS > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
for L in $LIBS $LIBS; do
  if [ $L = cur ]; then P=artes_amd/lib/libartes_hip.so; else P=artes_amd/lib/libartes_hip_$L.so; fi
  ARTES_LIB_PATH=$P timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variants > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', d['value'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done
PL=""; for L in $LIBS; do if [ $L = cur ]; then PL="$PL artes_amd/lib/libartes_hip.so"; else PL="$PL artes_amd/lib/libartes_hip_$L.so"; fi; done
timeout -k 10 300 bash tools/valu_ab.sh $T/valu ray3d 1e8 $PL > $O/valu.txt 2>&1 || { tail -5 $O/valu.txt; exit 1; }
grep "k_trace\|==" $O/valu.txt
[ -n "$NOTEST" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log

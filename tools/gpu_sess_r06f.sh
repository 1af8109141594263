#!/bin/bash
# Round-6 session f (development tool): the configs[3] launch knobs re-swept on the fused-step
# build, and the bench step with and without the det_ordered detector (its cost on the bench grid).
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 900 bash tools/gpu_cfg_variants.sh r06f/knobs cur:- cur:ARTES_STEPS=8 cur:ARTES_REFILL=20 cur:ARTES_REFILL=12 \
  cur:ARTES_GBATCH=4 cur:ARTES_GBATCH=16 cur:ARTES_HBATCH=6 cur:- > $O/knobs.txt 2>&1 || { tail -10 $O/knobs.txt; exit 1; }
grep "^\[" $O/knobs.txt
for t in none det_ordered=1 none det_ordered=1; do
  if [ $t = none ]; then A=""; else A="--tune $t"; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-variants $A > $O/bench_$t.json 2> $O/bench_$t.err || { tail -5 $O/bench_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$t.json')); print('$t', d['value'], d['ms_per_step'], d['engine']['kernels'], d['roofline']['pipeline']['kernels'])"
done

#!/bin/bash
# Round-6 session h (development tool): the k_event variant and reproducibility tests on the
# fixed-point detector accumulated in LDS, then its cost on the bench grid again.
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_event_variants.py tests/test_gpu_grids_and_repro.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for t in none det_ordered=1 none det_ordered=1; do
  if [ $t = none ]; then A=""; else A="--tune $t"; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-variants $A > $O/bench_$t.json 2> $O/bench_$t.err || { tail -5 $O/bench_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$t.json')); print('$t', d['value'], d['ms_per_step'], d['engine']['kernels'], {k: v['ms_per_step'] for k, v in d['roofline']['pipeline']['kernels'].items()})"
done

#!/bin/bash
# Round-6 session l (development tool): coarse-grid steps per iteration A/B (ARTES_COARSE_NREP 5 / 6
# builds against the shipping 4) on the cloudy calls; the bench line on the profiled build; the
# configs[3] counters and full 73-angle phase curve at 1e9 per call; configs[4] at 1e8 per call.
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 900 bash tools/gpu_cfg_variants.sh r06l/crep cur:- crep5:- crep6:- cur:- crep5:- crep6:- > $O/crep.txt 2>&1 || { tail -10 $O/crep.txt; exit 1; }
grep "^\[" $O/crep.txt
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_final.json')); print('bench', d['value'], d['roofline']['frac'], d['roofline']['traffic'], (d['roofline']['limiter'] or {}).get('valu_insts_per_crossing'))"
timeout -k 10 1200 bash tools/gpu_cfg3_pmc.sh r06l/c3 full > $O/cfg3.txt 2>&1 || { tail -10 $O/cfg3.txt; exit 1; }
tail -3 $O/cfg3.txt
timeout -k 10 300 python tools/config_runs.py $O/cfg4 --which 4 --packets 1e8 > $O/cfg4.log 2>&1 || { tail -5 $O/cfg4.log; exit 1; }
tail -1 $O/cfg4.log | cut -c1-400

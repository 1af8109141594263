#!/bin/bash
# Round-6 final evidence (development tool), on a build whose profiles/r06 summaries are in place:
# the bench line (traffic and limiter from those summaries), the configs[3] counters and full
# 73-angle phase curve at 1e9 per call, configs[4] at 1e8 per call.
# usage (via gpurun): bash tools/gpu_sess_r06p.sh <out>
set -o pipefail
O=gpurun_out/${1:-r06p}; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_final.json')); print('bench', d['value'], d['roofline']['frac'], d['roofline']['traffic'], (d['roofline']['limiter'] or {}).get('valu_insts_per_crossing'))"
timeout -k 10 1200 bash tools/gpu_cfg3_pmc.sh ${1:-r06p}/c3 full > $O/cfg3.txt 2>&1 || { tail -10 $O/cfg3.txt; exit 1; }
tail -3 $O/cfg3.txt
timeout -k 10 300 python tools/config_runs.py $O/cfg4 --which 4 --packets 1e8 > $O/cfg4.log 2>&1 || { tail -5 $O/cfg4.log; exit 1; }
tail -1 $O/cfg4.log | cut -c1-400

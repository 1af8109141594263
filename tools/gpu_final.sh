#!/bin/bash
# Round-end evidence on a build whose profiles/r03 summaries are already in place (development
# tool): the bench line (traffic and limiter filled from those summaries), the configs[3]
# subset at 1e9 packets per call and configs[4] at 1e8.
# usage (via gpurun): bash tools/gpu_final.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
cat $O/bench_final.json
timeout -k 10 900 python tools/config_runs.py $O/cfg3 --which 3 --packets 1e9 --phases 19 --lambdas 13 > $O/cfg3.log 2>&1 || { tail -5 $O/cfg3.log; exit 1; }
tail -1 $O/cfg3.log
timeout -k 10 300 python tools/config_runs.py $O/cfg4 --which 4 --packets 1e8 > $O/cfg4.log 2>&1 || { tail -5 $O/cfg4.log; exit 1; }
tail -1 $O/cfg4.log

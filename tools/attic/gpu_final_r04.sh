#!/bin/bash
# Round-end evidence on the final round-4 build, after its profiles/r04 summaries are committed:
# the configs[3] counter passes and the whole 73-angle phase curve at 1e9 per call
# (tools/gpu_cfg3_pmc.sh ... full), the bench line (traffic and limiter filled from the
# committed summaries of the same library) and configs[4]'s 100-wavelength thermal spectrum.
# usage (via gpurun): bash tools/gpu_final_r04.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
bash tools/gpu_cfg3_pmc.sh $1 full || exit 1
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
cat $O/bench_final.json
timeout -k 10 300 python tools/config_runs.py $O/cfg4 --which 4 --packets 1e8 > $O/cfg4.log 2>&1 || { tail -5 $O/cfg4.log; exit 1; }
tail -1 $O/cfg4.log

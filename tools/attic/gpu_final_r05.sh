#!/bin/bash
# Round-end evidence on the final round-5 build, after its profiles/r05 bench summaries
# (tools/gpu_round.sh) are committed: the bench line (traffic and limiter from those summaries
# of the same library), the configs[3] counter passes and the whole 73-angle phase curve at 1e9
# per call (tools/gpu_cfg3_pmc.sh ... full), configs[4]'s 100-wavelength thermal spectrum, and
# the k_trace lane accounting / region timing of the development builds.
# usage (via gpurun): bash tools/gpu_final_r05.sh <out>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
md5sum artes_amd/lib/libartes_hip.so > $O/lib_md5.txt
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { echo "bench failed"; tail -20 $O/bench_final.err; exit 1; }
cat $O/bench_final.json
bash tools/gpu_cfg3_pmc.sh $1 full || exit 1
timeout -k 10 300 python tools/config_runs.py $O/cfg4 --which 4 --packets 1e8 > $O/cfg4.log 2>&1 || { tail -5 $O/cfg4.log; exit 1; }
tail -1 $O/cfg4.log
bash tools/gpu_lanes_regions.sh $1/lanes 1e8 > $O/lanes_regions.txt 2>&1 || { tail -5 $O/lanes_regions.txt; exit 1; }
echo "lanes and regions done"

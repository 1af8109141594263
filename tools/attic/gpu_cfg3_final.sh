#!/bin/bash
# configs[3] counter passes on the final build (as tools/gpu_s2.sh) and the 8-rank gloo
# rehearsal of bench.py on one card (its stdout must be exactly one JSON line)
set -o pipefail
O=gpurun_out/cfg3f; mkdir -p $O
export TMPDIR=/tmp
CFG="python3 tools/config_runs.py $O/cfgrun --which 3 --packets 1e8 --phases 4 --lambdas 4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg3/trace -o run -- $CFG > $O/cfg3_trace.log 2>&1 || { tail -20 $O/cfg3_trace.log; exit 1; }
cp $O/cfgrun/configs3_cloudy.json $O/cfg3_runs.json
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d $O/cfg3/pmc_$tag -o run -- $CFG > $O/cfg3_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $O/cfg3_$tag.log; exit 1; }
done
python3 tools/pmc_cfg_summary.py $O/cfg3 $O/cfg3_runs.json $O/cfg3_pmc_summary.json > /dev/null && echo "cfg3 counters done"
ARTES_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 8 --packets 5e7 --steps 2 --warmup 1 > $O/rehearsal8.json 2> $O/rehearsal8.err || { tail -20 $O/rehearsal8.err; exit 1; }
wc -l $O/rehearsal8.json
cat $O/rehearsal8.json | cut -c1-400

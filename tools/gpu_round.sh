#!/bin/bash
# One GPU-box session: parity tests, the default bench line, and the rocprofv3 evidence
# (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) of a bench run.
# usage (via gpurun): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROF_ARGS="--no-cpu-baseline --no-parity --no-variants"   # exactly the timed bench transport: 1 warmup + 3 steps of 1e9 packets (the profiled run holds 4e9 packets)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_trace.json 2> $OUT/prof_trace.err || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof/pmc_fetch -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_fetch.json 2> $OUT/prof_fetch.err || { echo "fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof/pmc_write -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_write.json 2> $OUT/prof_write.err || { echo "write failed"; exit 1; }
python3 tools/pmc_summary.py $OUT/prof 4e9 $OUT/pmc_summary.json > /dev/null && echo "profiles done"
# VALU-issue evidence of the same command: two SQ passes (8 SQ + 2 GRBM counters at most per pass)
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/sq/p1 -o run -- python3 bench.py $PROF_ARGS > $OUT/sq1.json 2> $OUT/sq1.err || { echo "sq pass 1 failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq/p2 -o run -- python3 bench.py $PROF_ARGS > $OUT/sq2.json 2> $OUT/sq2.err || { echo "sq pass 2 failed"; exit 1; }
python3 tools/pmc_sq_summary.py $OUT/sq $OUT/pmc_sq_summary.json $OUT/sq1.json 4e9 > /dev/null && python3 tools/pmc_table.py $OUT/sq > $OUT/pmc_sq_table.txt && echo "sq passes done"

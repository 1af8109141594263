#!/bin/bash
# One GPU-box session: parity tests, the default bench line, and the rocprofv3 evidence
# (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes) of a bench run.
# usage (via gpurun): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PROF_ARGS="--no-cpu-baseline"   # the default bench command (3 steps + 1 warmup of 1e9 packets); the CPU leg launches no GPU kernels
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_trace.json 2> $OUT/prof_trace.err || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof/pmc_fetch -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_fetch.json 2> $OUT/prof_fetch.err || { echo "fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof/pmc_write -o run -- python3 bench.py $PROF_ARGS > $OUT/prof_write.json 2> $OUT/prof_write.err || { echo "write failed"; exit 1; }
python3 tools/pmc_summary.py $OUT/prof 4e9 $OUT/pmc_summary.json > /dev/null && echo "profiles done"

#!/bin/bash
# Round-6 closing checks (development tool) on the shipping build: __graft_entry__.smoke(); the bench's collective path
# at one rank over RCCL (ARTES_DIST_FORCE=1) and at two ranks sharing the box's one card over gloo (RCCL refuses two
# ranks on one device).
set -o pipefail
mkdir -p gpurun_out/r06y
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06y/smoke.log 2>&1 || { tail -20 gpurun_out/r06y/smoke.log; exit 1; }
tail -1 gpurun_out/r06y/smoke.log
ARTES_DIST_FORCE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-variants > gpurun_out/r06y/bench_1rank_rccl.json 2> gpurun_out/r06y/bench_1rank_rccl.err || { tail -20 gpurun_out/r06y/bench_1rank_rccl.err; exit 1; }
cut -c1-300 gpurun_out/r06y/bench_1rank_rccl.json
ARTES_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-variants > gpurun_out/r06y/bench_2rank.json 2> gpurun_out/r06y/bench_2rank.err || { tail -20 gpurun_out/r06y/bench_2rank.err; exit 1; }
cat gpurun_out/r06y/bench_2rank.json | cut -c1-400

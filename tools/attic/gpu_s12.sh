#!/bin/bash
set -o pipefail
O=gpurun_out/s12; mkdir -p $O
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_HBATCH=4" "ARTES_HBATCH=10" "ARTES_BATCH_MIN=8" "ARTES_BATCH_MIN=24" "ARTES_STATIC=40" "ARTES_STATIC=56" "ARTES_REFILL=40" "ARTES_BATCH=2"

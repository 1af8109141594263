#!/bin/bash
set -o pipefail
O=gpurun_out/s13; mkdir -p $O
bash tools/cfg_env_sweep.sh $O/sweep "" "ARTES_EVENT_P1_1024=1"

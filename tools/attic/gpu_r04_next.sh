#!/bin/bash
# Round 4's last information session (development): the k_trace region timing of the final
# build, and cloudy launch-knob candidates for the next round (the defaults are not changed).
set -o pipefail
bash tools/gpu_time_regions.sh r04n2/tr 1e8 || exit 1
bash tools/gpu_cfg_variants.sh r04n2/cv cur:- cur:ARTES_REFILL=16 cur:ARTES_GBATCH=12 cur:ARTES_HBATCH=8 cur:ARTES_STATIC=24 cur:ARTES_DGRAB=64 cur:-

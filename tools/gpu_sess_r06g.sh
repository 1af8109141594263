#!/bin/bash
# Round-6 session g (development tool): the GPU suite, then the configs[3] A/B of k_event's
# unpadded LDS tables (default) against the cumulative tables alone (event_ldsu = 0).
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu_cfg_variants.sh r06g/ldsu cur:- cur:ARTES_EVENT_LDSU=0 cur:- cur:ARTES_EVENT_LDSU=0 > $O/ldsu.txt 2>&1 || { tail -10 $O/ldsu.txt; exit 1; }
cat $O/ldsu.txt

#!/bin/bash
# the oblate trajectory case under the CHECKED build only (cell-index checks before every
# per-cell table read), without and with the LDS per-cell table
set -o pipefail
O=gpurun_out/s6; mkdir -p $O
D=$PWD/artes_amd/lib/libartes_hip_debug.so
ARTES_KLDS=0 ARTES_LIB_PATH=$D timeout -k 10 120 python tools/oblate_probe.py > $O/oblate_debug_global.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/oblate_debug_global.txt; [ $rc -eq 0 ] || exit $rc
ARTES_LIB_PATH=$D timeout -k 10 120 python tools/oblate_probe.py > $O/oblate_debug_klds.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/oblate_debug_klds.txt; [ $rc -eq 0 ] || exit $rc

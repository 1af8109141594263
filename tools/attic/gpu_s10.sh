#!/bin/bash
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 300 bash tools/valu_ab.sh s10v ray3d 1e8 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $O/valu.txt 2>&1 || { tail -5 $O/valu.txt; exit 1; }
grep "==\|k_trace\|k_event\|pkt/s" $O/valu.txt
QP_CHECK=0 timeout -k 10 500 bash tools/ab_run.sh 3e8 base cur base cur > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt

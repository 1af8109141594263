#!/bin/bash
# Latency / issue counters of the transport kernels (development tool): per config, three
# rocprofv3 --pmc passes over tools/prof_one.py, summarised by tools/pmc_lat.py.
# usage (via gpurun): bash tools/pmc_lat.sh <out dir> <config>:<packets> [...]
set -o pipefail
O=$1; shift; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F64 SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for spec in "$@"; do
  CFG=${spec%%:*}; N=${spec##*:}
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/$CFG/p$i -o run -- python3 tools/prof_one.py $CFG $N > $O/$CFG.p$i.log 2>&1 || { echo "$CFG pass $i failed"; tail -5 $O/$CFG.p$i.log; exit 1; }
  done
  grep "pkt/s" $O/$CFG.p1.log
  python3 tools/pmc_lat.py $O/$CFG
done

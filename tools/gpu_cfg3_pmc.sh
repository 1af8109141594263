#!/bin/bash
# configs[3] evidence on the current library: kernel trace + FETCH / WRITE / TCC+LDS / two SQ
# counter passes of the cloudy calls (4 phase angles + 4 wavelengths at 1e8 per call),
# summarised by tools/pmc_cfg_summary.py (records the library md5); optionally the whole
# 73-angle phase curve at wavelengths(1) at 1e9 packets per call.
# usage (via gpurun): bash tools/gpu_cfg3_pmc.sh <tag> [full]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
md5sum artes_amd/lib/libartes_hip.so > $O/lib_md5.txt
CFG="python3 tools/config_runs.py $O/cfgrun --which 3 --packets 1e8 --phases 4 --lambdas 4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg3/trace -o run -- $CFG > $O/cfg3_trace.log 2>&1 || { tail -20 $O/cfg3_trace.log; exit 1; }
cp $O/cfgrun/configs3_cloudy.json $O/cfg3_runs.json
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d $O/cfg3/pmc_$tag -o run -- $CFG > $O/cfg3_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $O/cfg3_$tag.log; exit 1; }
done
python3 tools/pmc_cfg_summary.py $O/cfg3 $O/cfg3_runs.json $O/configs3_pmc_summary.json > /dev/null && echo "cfg3 counters done"
cp $O/cfg3/trace/run_kernel_stats.csv $O/configs3_kernel_stats.csv 2>/dev/null || true
if [ "$2" = full ]; then
  timeout -k 10 600 python3 tools/config_runs.py $O/full --which 3 --packets 1e9 --lambdas 1 > $O/full.log 2>&1 || { echo "full phase curve failed"; tail -5 $O/full.log; exit 1; }
  tail -1 $O/full.log
fi

#!/bin/bash
# PC sampling (rocprofv3 host-trap, time based) of one engine run, to find where k_trace and
# k_event spend their waves' time instruction by instruction.
#   usage: bash tools/gpu_pcsample.sh <tag> [workload] [packets] [interval_us]
# Output: gpurun_out/<tag>/ (rocprofv3 csv files) and the list of available sampling configs.
set -o pipefail
tag=${1:-pcs}
wl=${2:-cloudy}
n=${3:-1e8}
iv=${4:-1}
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 60 rocprofv3 -L > "$out/list_avail.txt" 2>&1
echo "list-avail rc=$?"
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
    --pc-sampling-unit time --pc-sampling-interval "$iv" --output-format csv \
    -d "$out/prof" -o "$wl" -- python3 tools/prof_one.py "$wl" "$n" > "$out/run.log" 2>&1
rc=$?
echo "pc sampling rc=$rc"
tail -5 "$out/run.log"
find "$out/prof" -type f -printf '%s %p\n' 2>/dev/null | head -20
exit $rc

#!/bin/bash
# Round-4 session b: the GPU suite on the current library (new: the 2-rank HIP CLI test, the
# exact crossing counter), then a probe of rocprofv3's PC sampling (listing first).
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
md5sum artes_amd/lib/libartes_hip.so > $O/lib_md5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -s KILL 60 rocprofv3 -L > $O/rocprof_L.txt 2>&1; echo "list rc=$?"
grep -i -A12 "pc.samp" $O/rocprof_L.txt | head -60

set -o pipefail
O=gpurun_out/s1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
QP_CHECK=0 timeout -k 10 300 python tools/quick_perf.py 3e8 > $O/qp_rel.txt 2>&1 || exit 1
cat $O/qp_rel.txt
timeout -k 10 400 python tools/fault_repro.py artes_amd/lib/libartes_hip_nbf_debug.so artes_amd/lib/libartes_hip_debug.so artes_amd/lib/libartes_hip_nbf_old_debug.so > $O/fault.txt 2>&1; rc=$?; cat $O/fault.txt; [ $rc -eq 0 ] || exit $rc
ARTES_LIB_PATH=$PWD/artes_amd/lib/libartes_hip_nbf.so QP_CHECK=0 timeout -k 10 300 python tools/quick_perf.py 3e8 > $O/qp_nbf.txt 2>&1 || exit 1
cat $O/qp_nbf.txt

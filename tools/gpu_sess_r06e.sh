set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
bash tools/gpu_ab_r06.sh r06e 3e8 base cur > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v "^==.*early\|EARLY" $O/ab.txt | head -30
bash tools/valu_ab.sh r06e/valu ray3d 1e8 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $O/valu.txt 2>&1 || { tail -5 $O/valu.txt; exit 1; }
grep "k_trace\|ray3d 1000" $O/valu.txt
bash tools/valu_ab.sh r06e/valuc cloudy 3e7 artes_amd/lib/libartes_hip_base.so artes_amd/lib/libartes_hip.so > $O/valuc.txt 2>&1 || { tail -5 $O/valuc.txt; exit 1; }
grep "k_trace\|cloudy 3" $O/valuc.txt
bash tools/gpu_lds_layout_ab.sh r06e/lds cur cum1 cum2 > $O/lds.txt 2>&1 || { tail -10 $O/lds.txt; exit 1; }
cat $O/lds.txt

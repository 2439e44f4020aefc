# round 6: 2-wave workgroups for k_xspec_w2 (4 per CU, barriers of 2 waves)
export TMPDIR=/tmp
out=gpurun_out/ab_x2w; mkdir -p $out; st=$out/status.txt
PPFIT_LIB=varlib/libppfit_x2w2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_bench or c3_bench or fullshape" > $out/pytest_x2w2.log 2>&1
rc=$?; echo "tests(x2w2) rc=$rc $(tail -1 $out/pytest_x2w2.log)" >> $st
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh x2w "c2 c3" "base lib:varlib/libppfit_x2w2.so" 2

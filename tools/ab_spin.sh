# round 6: the whole GPU suite on the final build, then C4 with the
# spin-polled read-backs (default) against hipStreamSynchronize
export TMPDIR=/tmp
out=gpurun_out/ab_spin; mkdir -p $out; st=$out/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
TESTK= bash tools/ab.sh spc4 "c4 c2" "base lib:varlib/libppfit_nospin.so" 2

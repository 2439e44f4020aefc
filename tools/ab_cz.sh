# round 6: C4 guess brute grid as a chirp z-transform (default build) against
# the direct sums (PPF_GUESS_CZ=0), after the align / guess parity tests
export TMPDIR=/tmp
out=gpurun_out/ab_cz; mkdir -p $out; st=$out/status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "align or c4 or guess or phase_shift or gettoas" > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
TESTK= bash tools/ab.sh czc4 "c4" "base lib:varlib/libppfit_nocz.so" 3

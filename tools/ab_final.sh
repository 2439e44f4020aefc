# round 6: the whole GPU suite on the final build, then the GetTOAs and C4
# lines with the opt-in polling
export TMPDIR=/tmp
out=gpurun_out/ab_final; mkdir -p $out; st=$out/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $out/smoke.txt)" >> $st
[ $rc -eq 0 ] || exit $rc
TESTK= bash tools/ab.sh fin "gtps gt c4" "base" 2

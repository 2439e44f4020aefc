# round 6: the whole GPU suite and smoke on the tree as committed last
export TMPDIR=/tmp
out=gpurun_out/final9; mkdir -p $out; st=$out/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $out/smoke.txt)" >> $st
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $out/bench_c2.log 2>&1
rc=$?; echo "c2 rc=$rc $(python tools/show.py $out/bench_c2.log 2>/dev/null | head -1)" >> $st
echo end >> $st

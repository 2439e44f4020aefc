# round 6: the whole GPU suite, smoke and the C2 / C3 / C5 / C4 / GetTOAs lines on the last build
export TMPDIR=/tmp
out=gpurun_out/final7; mkdir -p $out; st=$out/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $out/smoke.txt)" >> $st
[ $rc -eq 0 ] || exit $rc
run() {   # name, args
  timeout -k 10 400 python bench.py $2 > $out/bench_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc $(python tools/show.py $out/bench_$1.log 2>/dev/null | head -1)" >> $st
  return $rc
}
run c2 "" && \
run c3 "--fit full --nsub 10000 --steps 3 --warmup 1" && \
run c5 "--fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 3 --warmup 1" && \
run c4 "--fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 50 --warmup 5" && \
run gtps "--fit gettoas --psrfits --steps 4 --warmup 1"
echo end >> $st

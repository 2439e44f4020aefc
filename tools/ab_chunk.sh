# round 6: the long-row noise tests, then C2 with the 10k sub-ints of a pass
# split into calls of --chunk sub-ints (X of a chunk of 100 fits the MALL)
export TMPDIR=/tmp
out=gpurun_out/ab_chunk; mkdir -p $out; st=$out/status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "noise" > $out/pytest.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
[ $rc -eq 0 ] || exit $rc
for c in 10000 1000 250 100; do
  timeout -k 10 300 python bench.py --cpu-sample 0 --chunk $c > $out/c2_chunk$c.json 2> $out/c2_chunk$c.err
  rc=$?; echo "chunk $c rc=$rc $(python tools/show.py $out/c2_chunk$c.json 2>/dev/null)" >> $st
  [ $rc -eq 0 ] || exit $rc
done
echo end >> $st

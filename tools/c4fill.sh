#!/bin/bash
# round 6: ppalign without the per-iteration zero fills (tests, C4 lines, kernel trace)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/c4fill; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "align or psrfits or dist" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 50 --warmup 5 --cpu-sample 0 > $out/c4_$r.log 2>&1 || exit 1
  python tools/show.py $out/c4_$r.log | head -1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/ks -o ks --output-format csv -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 10 --warmup 2 --cpu-sample 0 > $out/ks.log 2>&1

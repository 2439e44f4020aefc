#!/bin/bash
# C4 A/B of bench.py's template normalisation (bench_prev.py: HEAD's boolean
# indexing) and the k_dsum_w occupancy build on C2.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4new${rep}.log 2>&1
  timeout -k 10 200 python bench_prev.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4old${rep}.log 2>&1
  for v in new old; do echo "c4-$v-$rep $(grep '^{' gpurun_out/bench_c4${v}${rep}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'))")"; done
done
bash tools/ab_c2.sh d4

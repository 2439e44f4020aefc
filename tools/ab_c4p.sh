#!/bin/bash
# ppalign GPU tests, then C4 with the current ppalign vs the previous one
# (pulseportraiture_amd/_ppalign_prev.py through bench_prev.py), interleaved.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "align" --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_c4p.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_c4p.log; tail -3 gpurun_out/gpu_tests_c4p.log; exit 1; }
tail -1 gpurun_out/gpu_tests_c4p.log
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4p_new${rep}.log 2>&1
  timeout -k 10 200 python bench_prev.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4p_old${rep}.log 2>&1
  for v in new old; do echo "c4-$v-$rep $(grep '^{' gpurun_out/bench_c4p_${v}${rep}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'))")"; done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4n/ks -o ks --output-format csv -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 --steps 3 > gpurun_out/prof_c4n.log 2>&1
echo traced

#!/bin/bash
# ppalign GPU tests, then a kernel trace of the C4 bench (launch gaps).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "align" --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_c4.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_c4.log; tail -3 gpurun_out/gpu_tests_c4.log; exit 1; }
tail -1 gpurun_out/gpu_tests_c4.log
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4_t.log 2>&1
grep '^{' gpurun_out/bench_c4_t.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4n/ks -o ks --output-format csv -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 --steps 3 > gpurun_out/prof_c4n.log 2>&1
echo traced

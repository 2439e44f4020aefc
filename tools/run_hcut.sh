#!/bin/bash
# harmonic cutoff check: GPU tests, then C3 and C5 benches
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_hcut2.log 2>&1
timeout -k 10 200 python bench.py --cpu-sample 0 --fit full > gpurun_out/bench_c3_hcut2.log 2>&1
timeout -k 10 200 python bench.py --cpu-sample 0 --fit scat --nchan 16384 --nbin 1024 --nsub 500 --chunk 100 > gpurun_out/bench_c5_hcut2.log 2>&1

#!/bin/bash
# harmonic cutoff check: GPU tests, then C3 benches with and without it
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_hcut.log 2>&1
timeout -k 10 200 python bench.py --cpu-sample 0 --fit full > gpurun_out/bench_c3_hcut.log 2>&1
PPF_NO_HCUT=1 timeout -k 10 200 python bench.py --cpu-sample 0 --fit full > gpurun_out/bench_c3_nohcut.log 2>&1

#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_gcut.log 2>&1
timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/bench_c2_gcut.log 2>&1

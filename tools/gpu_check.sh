#!/bin/bash
# One GPU round: parity tests, bench, kernel stats.  usage: tools/gpu_check.sh TAG [bench args]
set -e
tag=${1:-run}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
timeout -k 10 200 python bench.py --cpu-sample 0 "$@" > gpurun_out/bench_$tag.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 "$@" > gpurun_out/prof_$tag.log 2>&1

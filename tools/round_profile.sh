#!/bin/bash
# Full GPU evidence run: parity tests, bench (with CPU baseline), rocprofv3
# kernel stats of the same bench command, FETCH_SIZE / WRITE_SIZE PMC passes.
# usage: tools/round_profile.sh TAG   -> gpurun_out/{gpu_tests,bench,prof,pmc_*}_TAG
set -e
tag=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 > gpurun_out/prof_$tag.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$tag -o f --output-format csv -- python3 bench.py --nsub 2500 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_fetch_$tag.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$tag -o w --output-format csv -- python3 bench.py --nsub 2500 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_write_$tag.log 2>&1

#!/bin/bash
# ppalign path: GPU align tests, align bench, rocprof of the align bench.
set -e
tag=${1:-a}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "align or gauss" > gpurun_out/gpu_tests_align_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_align_$tag.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_align_$tag -o run --output-format csv -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/prof_align_$tag.log 2>&1

#!/bin/bash
# GPU parity tests + kernel trace of a 2500-sub-int bench step: tools/quick_trace.sh TAG
set -e
tag=${1:-q}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/vt_$tag -o run --output-format csv -- python3 bench.py --nsub 2500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/vt_$tag.log 2>&1
tail -2 gpurun_out/gpu_tests_$tag.log
grep '^{' gpurun_out/vt_$tag.log | cut -c1-400

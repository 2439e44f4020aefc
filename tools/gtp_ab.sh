#!/bin/bash
# GetTOAs from 16-bit PSRFITS files: loader depth 1 vs 2 (interleaved), after
# the GPU tests of the PSRFITS and GetTOAs paths.  usage: tools/gtp_ab.sh TAG
set -e
tag=${1:-g}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_psrfits.py tests/test_gpu_fullshape.py tests/test_gpu_dist.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_$tag.log; tail -3 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
for rep in 1 2; do
  for d in 1 2 3; do
    PPF_LOAD_DEPTH=$d timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gtp_d${d}_${rep}_$tag.log 2>&1
    echo "depth $d rep $rep $(grep '^{' gpurun_out/bench_gtp_d${d}_${rep}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'))")"
  done
done

#!/bin/bash
# k_pass change check: GPU parity suite, C3 and C5 benches, C5 FETCH/WRITE.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-p}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 200 python bench.py --fit full --nsub 2500 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5_$tag.log 2>&1
for c in c3 c5; do grep '^{' gpurun_out/bench_${c}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r['traffic'], d['mean_passes_per_fit'])"; done
bash tools/prof.sh c5$tag --fit scat --nchan 16384 --nbin 1024 --nsub 100 > /dev/null

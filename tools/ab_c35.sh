#!/bin/bash
# GPU parity suite, then C5 and C3 for the default build and every varlib/
# build, interleaved twice.  usage: tools/ab_c35.sh TAG
set -e
tag=${1:-o}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_$tag.log; tail -3 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
libs="pulseportraiture_amd/lib/libppfit.so $(ls varlib/*.so 2>/dev/null || true)"
for rep in 1 2; do
  for lib in $libs; do
    v=$(basename $lib .so | sed 's/libppfit_\?//'); v=${v:-main}
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}${rep}_$tag.log 2>&1
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3${v}${rep}_$tag.log 2>&1
    for c in c5 c3; do
      echo "$c-$v-$rep $(grep '^{' gpurun_out/bench_${c}${v}${rep}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (k.get('dsum') or {}).get('avg_launch_ms'), (k.get('xspec') or {}).get('avg_launch_ms'), (k.get('pass') or {}).get('avg_launch_ms'))")"
    done
  done
done

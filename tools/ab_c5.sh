#!/bin/bash
# C5 A/B: default build vs every varlib/ build, interleaved twice.
set -e
tag=${1:-c}
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in pulseportraiture_amd/lib/libppfit.so varlib/*.so; do
    [ -f "$lib" ] || continue
    v=$(basename $lib .so | sed 's/libppfit_\?//'); v=${v:-main}
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}${rep}_$tag.log 2>&1
    echo "c5-$v-$rep $(grep '^{' gpurun_out/bench_c5${v}${rep}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (k.get('xspec') or {}).get('avg_launch_ms'), (k.get('pass') or {}).get('avg_launch_ms'))")"
  done
done

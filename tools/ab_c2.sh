#!/bin/bash
# C2 A/B: default build vs every varlib/ build, interleaved three times.
set -e
tag=${1:-a}
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in pulseportraiture_amd/lib/libppfit.so varlib/*.so; do
    [ -f "$lib" ] || continue
    v=$(basename $lib .so | sed 's/libppfit_\?//'); v=${v:-main}
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/bench_c2${v}${rep}_$tag.log 2>&1
    echo "c2-$v-$rep $(grep '^{' gpurun_out/bench_c2${v}${rep}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (k.get('dsum') or {}).get('avg_launch_ms'), (k.get('xmom') or {}).get('avg_launch_ms'))")"
  done
done

#!/bin/bash
# C2, C3 and C5 for the default build and every varlib/ build (one pass
# each; the bench lines go to gpurun_out/ab4_*).  usage: tools/ab_r4a.sh TAG
tag=${1:-a}
export TMPDIR=/tmp
mkdir -p gpurun_out
libs="pulseportraiture_amd/lib/libppfit.so $(ls varlib/*.so 2>/dev/null || true)"
for lib in $libs; do
  v=$(basename $lib .so | sed 's/libppfit_\?//'); v=${v:-main}
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/ab4_c2${v}_$tag.log 2>&1 || exit 1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/ab4_c3${v}_$tag.log 2>&1 || exit 1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ab4_c5${v}_$tag.log 2>&1 || exit 1
  for c in c2 c3 c5; do
    echo "$c-$v $(grep '^{' gpurun_out/ab4_${c}${v}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), {n: v.get('avg_launch_ms') for n, v in k.items()})")" | tee -a gpurun_out/ab4_summary_$tag.txt
  done
done

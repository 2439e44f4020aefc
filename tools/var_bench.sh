#!/bin/bash
# bench.py under several library variants: tools/var_bench.sh TAG "<bench args>" lib1.so [lib2.so ...]
# -> gpurun_out/vb_TAG_<name>.log (one JSON line each)
export TMPDIR=/tmp
tag=$1; args=$2; shift 2
for lib in "$@"; do
  name=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 240 python bench.py $args --cpu-sample 0 > gpurun_out/vb_${tag}_$name.log 2>&1 || { echo "FAIL $lib"; exit 1; }
  echo "$name $(grep '^{' gpurun_out/vb_${tag}_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'xmom %.3f ms' % d['kernels'].get('xmom', d['kernels'].get('xspec', {})).get('avg_launch_ms', 0), 'dsum %.3f' % d['kernels']['dsum']['avg_launch_ms'], d['stage_ms'])")"
done

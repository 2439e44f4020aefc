#!/bin/bash
# Time bench.py stages for each library variant: tools/run_variants.sh out.log lib1.so lib2.so ...
out=$1; shift
for lib in "$@"; do
  echo "== $lib" >> $out
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --nsub 5000 --steps 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['total_ms'] for k, v in d['stages'].items()}, d['mean_passes_per_fit'])" >> $out || { echo FAIL >> $out; exit 1; }
done

#!/bin/bash
# C4 (ppalign) timing + pass counts of every varlib/ build
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
for lib in varlib/*.so; do
  nm=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 > gpurun_out/va_${tag}_$nm.log 2>&1 || { echo "FAIL $nm"; tail -5 gpurun_out/va_${tag}_$nm.log; exit 1; }
  echo "$nm align $(grep '^{' gpurun_out/va_${tag}_$nm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['mean_passes_per_fit'], d['mean_evals_per_fit'], d['passes_hist'])")"
done

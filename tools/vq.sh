#!/bin/bash
# time the moment pass under the varlib/ builds (C2 shape, 10k sub-ints)
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
for lib in varlib/*.so; do
  nm=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --nsub 10000 --steps 2 --warmup 1 --passes 4 --cpu-sample 0 > gpurun_out/vq_${tag}_$nm.log 2>&1 || { echo "FAIL $nm"; tail -5 gpurun_out/vq_${tag}_$nm.log; exit 1; }
  echo "$nm $(grep '^{' gpurun_out/vq_${tag}_$nm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['mean_evals_per_fit'], d['dm_pull_rms'])")"
done

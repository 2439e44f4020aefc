#!/bin/bash
# scattering-fit timing (C3 shape, and C5 with C5=1) under the varlib/ builds
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
for lib in varlib/*.so; do
  nm=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit full --nsub 2500 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/vq3_${tag}_$nm.log 2>&1 || { echo "FAIL $nm"; tail -5 gpurun_out/vq3_${tag}_$nm.log; exit 1; }
  echo "C3 $nm $(grep '^{' gpurun_out/vq3_${tag}_$nm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['mean_evals_per_fit'], d['tau_pull_rms'])")"
  if [ "${C5:-0}" = 1 ]; then
    PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/vq5_${tag}_$nm.log 2>&1 || { echo "FAIL5 $nm"; exit 1; }
    echo "C5 $nm $(grep '^{' gpurun_out/vq5_${tag}_$nm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_ms'], d['mean_evals_per_fit'], d['tau_pull_rms'])")"
  fi
done

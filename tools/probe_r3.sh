#!/bin/bash
# Round-3 probe: k_tr_mom section profile on the C4 shape (PPF_TM_PROF
# build), C4 kernel statistics, and the A/B of varlib builds on C3/C5.
# usage: tools/probe_r3.sh TAG
set -e
tag=${1:-p}
export TMPDIR=/tmp
mkdir -p gpurun_out
c4="--fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0"
if [ -f varlib/libppfit_tprof.so ]; then
  PPFIT_LIB=varlib/libppfit_tprof.so timeout -k 10 200 python tools/tprof.py > gpurun_out/tprof_c4_$tag.log 2>&1
  PPFIT_LIB=varlib/libppfit_tprof.so timeout -k 10 200 python tools/tprof.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/tprof_c2_$tag.log 2>&1
  tail -8 gpurun_out/tprof_c4_$tag.log
  tail -8 gpurun_out/tprof_c2_$tag.log
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag/ks_c4 -o ks --output-format csv -- python3 bench.py $c4 --steps 3 > gpurun_out/prof_$tag.ks_c4.log 2>&1
vs=""
for lib in varlib/*.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so | sed 's/libppfit_//')
  [ $v = tprof ] && continue
  vs="$vs c3$v c5$v"
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3${v}_$tag.log 2>&1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}_$tag.log 2>&1
done
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5_$tag.log 2>&1
for c in c3 c5 $vs; do
  f=gpurun_out/bench_${c}_$tag.log
  [ -f $f ] || continue
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (d.get('roofline') or {}).get('frac'), (k.get('xspec') or {}).get('avg_launch_ms'))")"
done

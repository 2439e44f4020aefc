#!/bin/bash
# A/B of the spectrum kernels: the GPU parity suite on the default build,
# then C3/C5/C4 for the default build and every varlib/ build, and the
# PSRFITS GetTOAs path with and without the overlapped read/upload.
# usage: tools/ab_r3d.sh TAG
set -e
tag=${1:-d}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_$tag.log; tail -3 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
run() {   # name lib
  local v=$1 lib=$2
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3${v}_$tag.log 2>&1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}_$tag.log 2>&1
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4${v}_$tag.log 2>&1
}
run "" pulseportraiture_amd/lib/libppfit.so
vs=""
for lib in varlib/*.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so | sed 's/libppfit_//')
  vs="$vs $v"
  run $v $lib
done
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gtp_$tag.log 2>&1
PPF_PSRFITS_OVERLAP=0 timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gtpnoov_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gtp2_$tag.log 2>&1
for v in "" $vs; do
  for c in c3 c5 c4; do
    f=gpurun_out/bench_${c}${v}_$tag.log
    echo "$c${v:+-$v} $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (k.get('xspec') or {}).get('avg_launch_ms'), (d.get('parity') or {}).get('ok'))")"
  done
done
for c in gtp gtpnoov gtp2; do
  echo "$c $(grep '^{' gpurun_out/bench_${c}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'))")"
done

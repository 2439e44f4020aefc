#!/bin/bash
# Round-3 evidence run: full GPU parity suite, then every bench line (C2
# headline, single-call latency, C3 at its real per-GPU share with the
# Newton and the scipy-path solvers, C5, C4, GetTOAs end to end from host
# float32 archives and from 16-bit PSRFITS files).  Each step has its own
# time limit; a failing test run stops the script.
# usage: tools/evid_r3.sh TAG [tests|notests]
set -e
tag=${1:-a}
mode=${2:-tests}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$mode" = tests ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_$tag.log; tail -3 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_c2_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit single --cpu-sample 1 > gpurun_out/bench_single_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 2 > gpurun_out/bench_c3_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 --solver scipy > gpurun_out/bench_c3scipy_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 1 > gpurun_out/bench_c5_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 > gpurun_out/bench_gettoas_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gettoaspsrfits_$tag.log 2>&1
# A/B of any experimental builds in varlib/ (tools/build_variant.sh) on C3/C5
vs=""
for lib in varlib/*.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so | sed 's/libppfit_//')
  vs="$vs c2$v c3$v c5$v"
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/bench_c2${v}_$tag.log 2>&1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3${v}_$tag.log 2>&1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5${v}_$tag.log 2>&1
done
for c in c2 single c3 c3scipy c5 c4 gettoas gettoaspsrfits $vs; do
  f=gpurun_out/bench_${c}_$tag.log
  [ -f $f ] || continue
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), d.get('mean_passes_per_fit'), d.get('mean_evals_per_fit'), (d.get('roofline') or {}).get('frac'), (k.get('xspec') or {}).get('avg_launch_ms'), (d.get('parity') or {}).get('ok'))")"
done

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
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log | grep -v "^Approx"; exit 1; }
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
for c in c2 single c3 c3scipy c5 c4 gettoas gettoaspsrfits; do
  f=gpurun_out/bench_${c}_$tag.log
  [ -f $f ] || continue
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), d.get('mean_passes_per_fit'), d.get('mean_evals_per_fit'), (d.get('roofline') or {}).get('frac'), (d.get('parity') or {}).get('ok'))")"
done

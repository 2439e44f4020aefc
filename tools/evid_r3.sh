#!/bin/bash
# Round-3 evidence run: GPU parity suite, headline bench, single-call latency,
# C3 at its real per-GPU share (configs[2]: 80k / 8 = 10k sub-ints), and
# optionally the other configs.  usage: tools/evid_r3.sh TAG [quick|full]
set -e
tag=${1:-a}
mode=${2:-quick}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_c2_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit single --cpu-sample 1 > gpurun_out/bench_single_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 > gpurun_out/bench_c3_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 --solver scipy > gpurun_out/bench_c3scipy_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 1 > gpurun_out/bench_c5_$tag.log 2>&1
if [ "$mode" = full ]; then
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 > gpurun_out/prof_c2_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 > gpurun_out/bench_gettoas_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --pinned > gpurun_out/bench_gettoaspinned_$tag.log 2>&1
fi
for c in c2 single c3 c3scipy c5 c4 gettoas gettoaspinned; do
  f=gpurun_out/bench_${c}_$tag.log
  [ -f $f ] || continue
  echo "$c $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), (d.get('roofline') or {}).get('frac'), (d.get('fp64_roofline') or {}).get('frac'), (d.get('parity') or {}).get('ok'))")"
done

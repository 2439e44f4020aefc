#!/bin/bash
# Round-2 evidence run: GPU parity suite, headline bench (with CPU baseline +
# parity), rocprof kernel stats of the same command, FETCH/WRITE passes, and
# the other configs (C3 with and without the harmonic cutoff, C5, C4,
# GetTOAs end to end).
set -e
tag=${1:-f}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_c2_$tag.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$tag -o run --output-format csv -- python3 bench.py --cpu-sample 0 > gpurun_out/prof_c2_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit full --nsub 2500 --steps 3 --warmup 1 > gpurun_out/bench_c3_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit full --nsub 2500 --steps 3 --warmup 1 --cpu-sample 0 --no-hcut > gpurun_out/bench_c3nohcut_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 1 > gpurun_out/bench_c5_$tag.log 2>&1
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --cpu-sample 0 > gpurun_out/bench_c4_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 > gpurun_out/bench_gettoas_$tag.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --pinned > gpurun_out/bench_gettoaspinned_$tag.log 2>&1
bash tools/prof.sh c2$tag --nsub 2500 --passes 1 > /dev/null
for c in c2 c3 c3nohcut c5 c4 gettoas gettoaspinned; do echo "$c $(grep '^{' gpurun_out/bench_${c}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), (d.get('roofline') or {}).get('frac'), (d.get('fp64_roofline') or {}).get('frac'), (d.get('parity') or {}).get('ok'))")"; done

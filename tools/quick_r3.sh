set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_q.log 2>&1 || { grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_q.log; tail -3 gpurun_out/gpu_tests_q.log; exit 1; }
tail -1 gpurun_out/gpu_tests_q.log
timeout -k 10 300 python bench.py --fit full --nsub 10000 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3_q.log 2>&1
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c5_q.log 2>&1
timeout -k 10 300 python bench.py --fit gettoas --steps 2 --warmup 1 --psrfits > gpurun_out/bench_gettoaspsrfits_q.log 2>&1
timeout -k 10 300 python tools/psrfits_prof.py 8 > gpurun_out/psrfits_prof_q.log 2>&1
for c in c3 c5 gettoaspsrfits; do echo "$c $(grep '^{' gpurun_out/bench_${c}_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), (k.get('xspec') or {}).get('avg_launch_ms'))")"; done
head -5 gpurun_out/psrfits_prof_q.log

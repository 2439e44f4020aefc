set -e
TAG=${1:-s}
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s1.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --chunk 100 --steps 2 --warmup 1 > gpurun_out/bench_scat_$TAG.log 2>&1
timeout -k 10 300 python bench.py --fit full --nsub 2500 --steps 2 --warmup 1 > gpurun_out/bench_full_$TAG.log 2>&1

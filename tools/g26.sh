# block-FFT kernels templated on the mixed-radix flag: GPU suite, then C4,
# single-call latency, nbin 1000 and C2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g26_pytest.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g26_c4.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --fit single --cpu-sample 0 > gpurun_out/g26_single.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --nbin 1000 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g26_nb1000.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g26_c2.log 2>&1 || exit 3
for f in c4 single nb1000 c2; do echo "$f $(python tools/show.py gpurun_out/g26_$f.log | head -1)"; done

cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --mom-x > gpurun_out/g3_c2_momx.json 2> gpurun_out/g3_c2_momx.err &&
timeout -k 10 300 python bench.py --fit full --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/g3_c3.json 2> gpurun_out/g3_c3.err &&
timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/g3_c5.json 2> gpurun_out/g3_c5.err &&
timeout -k 10 300 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g3_c4.json 2> gpurun_out/g3_c4.err &&
(timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g3_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/g3_status.txt)
echo "end rc=$?" >> gpurun_out/g3_status.txt

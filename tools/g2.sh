cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ok() { rc=$?; echo "$1 rc=$rc" >> gpurun_out/g2_status.txt; [ $rc -le 1 ]; }
(timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g2_tests.log 2>&1; ok tests) &&
(timeout -k 10 600 env PPF_MOM_X=1 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g2_momx_tests.log 2>&1; ok momx_tests) &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g2_c2_base.json 2> gpurun_out/g2_c2_base.err &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --mom-x > gpurun_out/g2_c2_momx.json 2> gpurun_out/g2_c2_momx.err &&
timeout -k 10 300 python bench.py --fit full --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/g2_c3.json 2> gpurun_out/g2_c3.err
echo "end rc=$?" >> gpurun_out/g2_status.txt

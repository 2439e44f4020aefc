cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
(timeout -k 10 400 env PPF_MOM_X=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -x -q --timeout 120 --timeout-method thread > gpurun_out/momx_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ]) &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/c2_base.json 2> gpurun_out/c2_base.err &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --mom-x > gpurun_out/c2_momx.json 2> gpurun_out/c2_momx.err

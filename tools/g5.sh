cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_psrfits.py tests/test_gpu_parity.py tests/test_gpu_fullshape.py -m gpu -x -q --timeout 120 --timeout-method thread -k "psrfits or gettoas or get_toas or getoas" > gpurun_out/g5_pytest.log 2>&1 &&
timeout -k 10 400 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g5_tl_psrfits.json > gpurun_out/g5_gt_psrfits.json 2> gpurun_out/g5_gt_psrfits.err &&
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g5_c2.json 2> gpurun_out/g5_c2.err
echo "end rc=$?" >> gpurun_out/g5_status.txt

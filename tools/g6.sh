cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g6_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/g6_status.txt
# only ordinary test failures (1) let the profile run follow
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/g6_prof -o gt -- python3 bench.py --fit gettoas --psrfits --steps 1 --warmup 1 > gpurun_out/g6_gt.json 2> gpurun_out/g6_gt.err
echo "end rc=$?" >> gpurun_out/g6_status.txt
fi

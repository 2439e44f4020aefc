cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g8_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/g8_status.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g8_tl_psrfits.json > gpurun_out/g8_gt_psrfits.json 2> gpurun_out/g8_gt_psrfits.err || exit 2
echo "gettoas ok" >> gpurun_out/g8_status.txt
bash tools/ab_r4a.sh g8
echo "end rc=$?" >> gpurun_out/g8_status.txt

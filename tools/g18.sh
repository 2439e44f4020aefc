cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g18_pytest.log 2>&1 || exit 2
for rep in 1 2; do
timeout -k 10 300 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g18_tl_$rep.json > gpurun_out/g18_gt_$rep.json 2> gpurun_out/g18_gt_$rep.err || exit 3
done
echo end

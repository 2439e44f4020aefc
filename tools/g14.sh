cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g14_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/g14_status.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
timeout -k 10 300 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g14_tl_$rep.json > gpurun_out/g14_gt_$rep.json 2> gpurun_out/g14_gt_$rep.err || exit 2
echo "gt $rep $(python tools/show.py gpurun_out/g14_gt_$rep.json | head -1)" >> gpurun_out/g14_status.txt
done
timeout -k 10 300 python bench.py --fit gettoas --steps 3 --warmup 1 > gpurun_out/g14_gtf32.json 2> gpurun_out/g14_gtf32.err || exit 3
echo "gt f32 $(python tools/show.py gpurun_out/g14_gtf32.json | head -1)" >> gpurun_out/g14_status.txt
echo end >> gpurun_out/g14_status.txt

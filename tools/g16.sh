cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "psrfits or load_data or get_toas or noise" > gpurun_out/g16_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/g16_pytest.log)" >> gpurun_out/g16_status.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
timeout -k 10 300 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g16_tl_$rep.json > gpurun_out/g16_gt_$rep.json 2> gpurun_out/g16_gt_$rep.err || exit 2
echo "gt $rep $(python tools/show.py gpurun_out/g16_gt_$rep.json | head -1)" >> gpurun_out/g16_status.txt
done
bash tools/g15.sh
echo end >> gpurun_out/g16_status.txt

# pinned-slot budget change: PSRFITS GPU tests, GetTOAs from PSRFITS twice
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "psrfits or get_toas or gettoas or stager or pinned" > gpurun_out/g29_pytest.log 2>&1 || exit 2
for rep in 1 2; do
timeout -k 10 200 python bench.py --fit gettoas --psrfits --steps 4 --warmup 1 > gpurun_out/g29_gt_$rep.json 2> gpurun_out/g29_gt_$rep.err || exit 3
echo "gt $rep $(python -c "import json; d=json.loads(open('gpurun_out/g29_gt_$rep.json').readline()); print(d['value'])")"
done

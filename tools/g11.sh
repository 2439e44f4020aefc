cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g11_pytest.log 2>&1 || exit 1
for v in "base" "PPF_LOAD_DEPTH=2" "PPF_READ_THREADS=16" "PPF_LOAD_AHEAD=1"; do
  e=""; [ "$v" != base ] && e="$v"
  timeout -k 10 300 env $e python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g11_tl_${v%%=*}.json > gpurun_out/g11_gt_${v%%=*}.json 2> gpurun_out/g11_gt_${v%%=*}.err || exit 2
  echo "$v $(python tools/show.py gpurun_out/g11_gt_${v%%=*}.json)" >> gpurun_out/g11_status.txt
done
echo "end" >> gpurun_out/g11_status.txt

# GetTOAs loader: kernel-staged fit inputs (PPF_STAGE_KERNEL 1 / 0), loads
# ahead 3 with 4 pinned slots (candidate defaults), A/B in ONE call
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psrfits.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "psrfits or copy_from_pinned or stager or get_toas or gettoas or fit_batch or full" > gpurun_out/g22_pytest.log 2>&1 || exit 2
for rep in 1 2 3; do
for v in k1 k0; do
  case $v in
    k1) e="PPF_STAGE_KERNEL=1 PPF_LOAD_AHEAD=3 PPF_PINNED_SLOTS=4" ;;
    k0) e="PPF_STAGE_KERNEL=0 PPF_LOAD_AHEAD=3 PPF_PINNED_SLOTS=4" ;;
  esac
  env $e timeout -k 10 200 python bench.py --fit gettoas --psrfits --steps 4 --warmup 1 --timeline gpurun_out/g22_tl_${v}_$rep.json > gpurun_out/g22_gt_${v}_$rep.json 2> gpurun_out/g22_gt_${v}_$rep.err || exit 3
  echo "$v $rep $(python -c "import json; d=json.loads(open('gpurun_out/g22_gt_${v}_$rep.json').readline()); print(d['value'])")" | tee -a gpurun_out/g22_status.txt
done
done
echo end

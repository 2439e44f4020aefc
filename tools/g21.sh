# A/B of the GetTOAs loader in ONE call: upload and unpack on separate
# streams (this build); pinned slots 2 / 3 and loads ahead 2 / 3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g21_pytest.log 2>&1 || exit 2
for rep in 1 2 3; do
for v in base s2 a3 a3s4; do
  case $v in
    base) e="PPF_PINNED_SLOTS=3" ;;
    s2) e="PPF_PINNED_SLOTS=2" ;;
    a3) e="PPF_LOAD_AHEAD=3" ;;
    a3s4) e="PPF_LOAD_AHEAD=3 PPF_PINNED_SLOTS=4" ;;
  esac
  env $e timeout -k 10 200 python bench.py --fit gettoas --psrfits --steps 4 --warmup 1 --timeline gpurun_out/g21_tl_${v}_$rep.json > gpurun_out/g21_gt_${v}_$rep.json 2> gpurun_out/g21_gt_${v}_$rep.err || exit 3
  echo "$v $rep $(python -c "import json; d=json.loads(open('gpurun_out/g21_gt_${v}_$rep.json').readline()); print(d['value'])")" | tee -a gpurun_out/g21_status.txt
done
done
echo end

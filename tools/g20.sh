# A/B of the GetTOAs loader options in ONE call (box-to-box spread ~10 %):
# native reader (this build) with the queue thread on / off and the
# interpreter switch interval at its default 5 ms / 1 ms / 0.5 ms
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_psrfits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g20_pytest.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/psrfits_bw.py 6 > gpurun_out/g20_bw.log 2>&1 || exit 2
for rep in 1 2 3; do
for v in q1 q0 q1s1 q1s05; do
  case $v in
    q1) e="PPF_QUEUE_THREAD=1" ;;
    q0) e="PPF_QUEUE_THREAD=0" ;;
    q1s1) e="PPF_QUEUE_THREAD=1 PPF_SWITCH_INTERVAL_MS=1" ;;
    q1s05) e="PPF_QUEUE_THREAD=1 PPF_SWITCH_INTERVAL_MS=0.5" ;;
  esac
  env $e timeout -k 10 200 python bench.py --fit gettoas --psrfits --steps 4 --warmup 1 --timeline gpurun_out/g20_tl_${v}_$rep.json > gpurun_out/g20_gt_${v}_$rep.json 2> gpurun_out/g20_gt_${v}_$rep.err || exit 3
  echo "$v $rep $(python -c "import json; d=json.loads(open('gpurun_out/g20_gt_${v}_$rep.json').readline()); print(d['value'])")" | tee -a gpurun_out/g20_status.txt
done
done
echo end

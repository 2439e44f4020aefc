# A/B of the PSRFITS loader options in ONE call (box-to-box spread is ~10 %)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for v in q1 q0 q1c0 q1c64; do
  case $v in
    q1) e="PPF_QUEUE_THREAD=1" ;;
    q0) e="PPF_QUEUE_THREAD=0" ;;
    q1c0) e="PPF_QUEUE_THREAD=1 PPF_UPLOAD_CHUNK_MB=0" ;;
    q1c64) e="PPF_QUEUE_THREAD=1 PPF_UPLOAD_CHUNK_MB=64" ;;
  esac
  env $e timeout -k 10 200 python bench.py --fit gettoas --psrfits --steps 3 --warmup 1 --timeline gpurun_out/g19_tl_${v}_$rep.json > gpurun_out/g19_gt_${v}_$rep.json 2> gpurun_out/g19_gt_${v}_$rep.err || exit 3
  echo "$v $rep $(python -c "import json; d=json.loads(open('gpurun_out/g19_gt_${v}_$rep.json').readline()); print(d['value'])")" | tee -a gpurun_out/g19_status.txt
done
done
echo end

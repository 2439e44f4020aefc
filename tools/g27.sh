# k_postfit with one wave per sub-int (main, PPF_POSTFIT_PB=64) vs the
# 256-thread layout (varlib pb256): GPU suite, then C2 / C3 / C5, two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g27_pytest.log 2>&1 || exit 2
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_pb256.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g27_c2_${v}_$rep.log 2>&1 || exit 3
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit full --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g27_c3_${v}_$rep.log 2>&1 || exit 3
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g27_c5_${v}_$rep.log 2>&1 || exit 3
  for c in c2 c3 c5; do
  echo "$c $v $rep $(grep '^{' gpurun_out/g27_${c}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), d.get('stage_ms'))")" | tee -a gpurun_out/g27_status.txt
  done
done
done
echo end

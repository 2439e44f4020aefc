# k_pass without the end-of-row selects in whole iterations (main) vs the
# masked loop (varlib mask): GPU suite, then C3 and C5 A/B, two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g25_pytest.log 2>&1 || exit 2
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_mask.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit full --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g25_c3_${v}_$rep.log 2>&1 || exit 3
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g25_c5_${v}_$rep.log 2>&1 || exit 3
  for c in c3 c5; do
  echo "$c $v $rep $(grep '^{' gpurun_out/g25_${c}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), {n: v.get('avg_launch_ms') for n, v in k.items()})")" | tee -a gpurun_out/g25_status.txt
  done
done
done
echo end

# trust-region step with a lane per sub-int (main, k_tr_step_l + k_tr_gates)
# vs a wave per sub-int (varlib tsw): GPU suite, then C3 / C5, two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g33_pytest.log 2>&1 || exit 2
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_tsw.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit full --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g33_c3_${v}_$rep.log 2>&1 || exit 3
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g33_c5_${v}_$rep.log 2>&1 || exit 3
  for c in c3 c5; do
  echo "$c $v $rep $(grep '^{' gpurun_out/g33_${c}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), d.get('stage_ms'), d.get('evaluations_per_fit'), d.get('passes_per_fit'))")" | tee -a gpurun_out/g33_status.txt
  done
done
done
echo end

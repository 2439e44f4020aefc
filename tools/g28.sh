# k_tr_mom with one wave per sub-int (main, up to 2048 channels) vs the
# 256-thread layout (varlib tm256): GPU suite, then C2 and C4, two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g28_pytest.log 2>&1 || exit 2
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_tm256.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g28_c2_${v}_$rep.log 2>&1 || exit 3
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g28_c4_${v}_$rep.log 2>&1 || exit 3
  for c in c2 c4; do
  echo "$c $v $rep $(grep '^{' gpurun_out/g28_${c}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), d.get('stage_ms'))")" | tee -a gpurun_out/g28_status.txt
  done
done
done
echo end

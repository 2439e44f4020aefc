# k_guess fused-mode harmonic limit (main build) + GPU parity subset, then
# C2 A/B main vs k_moments KU=8 (varlib/libppfit_mku2.so), two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g23_pytest.log 2>&1 || exit 2
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_mku2.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --steps 4 --warmup 1 > gpurun_out/g23_c2_${v}_$rep.log 2>&1 || exit 3
  echo "$v $rep $(grep '^{' gpurun_out/g23_c2_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], d.get('ms_per_step'), {n: v.get('avg_launch_ms') for n, v in k.items()})")" | tee -a gpurun_out/g23_status.txt
done
done
echo end

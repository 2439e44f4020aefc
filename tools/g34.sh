# k_xspec_w<10> model pairs loaded ahead: 4 (main) vs 2 vs 6, C2, two reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_mp2.so varlib/libppfit_mp6.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/g34_c2_${v}_$rep.log 2>&1 || exit 3
  echo "c2 $v $rep $(grep '^{' gpurun_out/g34_c2_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], {n: v.get('avg_launch_ms') for n, v in k.items()})")"
done
done

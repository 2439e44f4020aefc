# occupancy sensitivity of k_xspec_w<10> at C2: 4-wave workgroups (main,
# two per CU = 2 waves/SIMD), 2-wave (three per CU = 1.5 waves/SIMD), 8-wave
# (one per CU = 2 waves/SIMD, one 8-wave barrier per round)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_xw2.so varlib/libppfit_xw8.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 200 python bench.py --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/g30_c2_$v.log 2>&1 || exit 3
  echo "c2 $v $(grep '^{' gpurun_out/g30_c2_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels') or {}; print(d['value'], {n: v.get('avg_launch_ms') for n, v in k.items()})")"
done

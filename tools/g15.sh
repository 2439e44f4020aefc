cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_pass2k6.so; do
  v=$(basename $lib .so)
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit full --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/g15_c3_${v}_$rep.json 2> gpurun_out/g15_c3_${v}_$rep.err || exit 1
  PPFIT_LIB=$lib timeout -k 10 300 python bench.py --fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g15_c5_${v}_$rep.json 2> gpurun_out/g15_c5_${v}_$rep.err || exit 2
  echo "c3 $v $rep $(python tools/show.py gpurun_out/g15_c3_${v}_$rep.json | tr '\n' ' ')" >> gpurun_out/g15_status.txt
  echo "c5 $v $rep $(python tools/show.py gpurun_out/g15_c5_${v}_$rep.json | tr '\n' ' ')" >> gpurun_out/g15_status.txt
done
done
echo end >> gpurun_out/g15_status.txt

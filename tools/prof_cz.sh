# round 6: kernel trace of C4 with / without the chirp z-transform guess grid
export TMPDIR=/tmp
out=gpurun_out/czprof; mkdir -p $out
for v in base nocz; do
  if [ $v = base ]; then L=pulseportraiture_amd/lib/libppfit.so; else L=varlib/libppfit_$v.so; fi
  PPFIT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o $v -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 10 --warmup 2 --cpu-sample 0 > $out/$v.log 2>&1 || exit 1
  echo "$v done" >> $out/status.txt
done

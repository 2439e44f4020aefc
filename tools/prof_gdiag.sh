# round 6 (timing only): k_guess at C4 with the brute grid / polish removed
export TMPDIR=/tmp
out=gpurun_out/gdiag; mkdir -p $out
for v in base gdiag1 gdiag3; do
  if [ $v = base ]; then L=pulseportraiture_amd/lib/libppfit.so; else L=varlib/libppfit_$v.so; fi
  PPFIT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$v -o $v -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 10 --warmup 2 --cpu-sample 0 > $out/$v.log 2>&1 || exit 1
  echo "$v done" >> $out/status.txt
done

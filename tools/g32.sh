# half-buffer wave FFT with part of the next row prefetched (PF 4 / 8 of 16
# loads per lane) vs none vs k_noise_w; output digests must match
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_nh3.so varlib/libppfit_pf4.so varlib/libppfit_pf8.so; do
  PPFIT_LIB=$lib timeout -k 10 120 python tools/noise_bench.py || exit 3
done
done

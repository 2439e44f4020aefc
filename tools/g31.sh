# half-buffer wave FFT prototype (k_noise_h) vs k_noise_w: 327,680 rows of
# 2048 bins, event-timed, output digests must match
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in pulseportraiture_amd/lib/libppfit.so varlib/libppfit_nh3.so varlib/libppfit_nh4.so; do
  PPFIT_LIB=$lib timeout -k 10 120 python tools/noise_bench.py || exit 3
done

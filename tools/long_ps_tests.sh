# round 6: FFTFIT past the LDS transforms, then the FFTFIT / narrowband suite
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "phase_shift or narrowband" > gpurun_out/long_ps_tests.log 2>&1
rc=$?; tail -12 gpurun_out/long_ps_tests.log; exit $rc

# round 6: fits at nbin past the LDS transforms, then the rest of the fit suite
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "16384 or 10002 or 8193" > gpurun_out/long_fit_tests.log 2>&1
rc=$?; tail -8 gpurun_out/long_fit_tests.log; exit $rc

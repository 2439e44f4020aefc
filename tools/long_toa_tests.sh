# round 6: GetTOAs and fits at nbin past the LDS transforms
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "16384 or 10002 or 8193 or gettoas_matches or gauss" > gpurun_out/long_toa_tests.log 2>&1
rc=$?; tail -12 gpurun_out/long_toa_tests.log; exit $rc

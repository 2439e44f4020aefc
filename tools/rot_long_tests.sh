# round 6: rotation / noise tests incl. the long-row transforms
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rotate or noise" > gpurun_out/rot_long_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rot_long_tests.log; exit $rc

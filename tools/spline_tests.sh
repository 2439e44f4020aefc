#!/bin/bash
# round 6: spline templates resampled to lengths that are not powers of two
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fullshape.py -k "spline" > gpurun_out/spline.log 2>&1
rc=$?
tail -20 gpurun_out/spline.log
exit $rc

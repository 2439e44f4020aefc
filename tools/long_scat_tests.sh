#!/bin/bash
# round 6: scattered Gaussian portraits on long rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_gauss_portraits_long_scattered_match_oracle" \
  "tests/test_gpu_parity.py::test_gauss_portraits_match_reference" \
  "tests/test_gpu_parity.py" -k "gauss or rotate or long or chi2 or zap" \
  > gpurun_out/long_scat.log 2>&1
rc=$?
tail -25 gpurun_out/long_scat.log
exit $rc

#!/bin/bash
# round 6: GetTOAs with a scattered .gmodel on long rows vs the reference
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_gettoas_branches_match_reference[scatlong]" \
  "tests/test_gpu_fullshape.py::test_gettoas_branches_match_reference[scatgm]" \
  "tests/test_gpu_fullshape.py::test_fullshape_gettoas_matches_reference[long16384]" \
  > gpurun_out/scatlong.log 2>&1
rc=$?
tail -25 gpurun_out/scatlong.log
exit $rc

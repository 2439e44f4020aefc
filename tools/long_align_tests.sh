#!/bin/bash
# round 6: FFTFIT grids in global memory (Ns = nbin), ppalign at long rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_fit_phase_shift_long_rows_match_oracle" \
  "tests/test_gpu_fullshape.py::test_align_long_rows_match_oracle" \
  "tests/test_gpu_fullshape.py::test_fullshape_align_matches_reference" \
  > gpurun_out/long_align.log 2>&1
rc=$?
tail -15 gpurun_out/long_align.log
exit $rc

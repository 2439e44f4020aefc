#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag_long_align3.py 2048 8192 > gpurun_out/diag_long_align2.log 2>&1
rc=$?
tail -30 gpurun_out/diag_long_align2.log
exit $rc

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 0.1" "32 0.5" "32 0.2"; do
  set -- $cfg
  NCH=$1 NOISE=$2 timeout -k 10 300 python -u tools/diag_long_align.py 2048 8192 16384 >> gpurun_out/diag_long_align.log 2>&1 || { tail -20 gpurun_out/diag_long_align.log; exit 1; }
done
grep nbin gpurun_out/diag_long_align.log

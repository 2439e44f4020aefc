#!/bin/bash
# k_xmom_g sensitivity: section cycle profile (xprof build) + bench under
# base / no-FFT / no-MFMA builds (timing only; the latter two fit garbage).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
PPFIT_LIB=varlib/libppfit_xprof.so timeout -k 10 200 python tools/xprof.py > gpurun_out/xprof_$1.log 2>&1
bash tools/var_bench.sh $1 "--nsub 2500 --steps 2 --warmup 1 --passes 2" varlib/libppfit_*.so > gpurun_out/sens_$1.log 2>&1

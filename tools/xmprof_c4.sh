#!/bin/bash
# Section cycle profile of k_xmom_g<9> at C4 from the PPF_XM_PROF build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PPFIT_LIB=$PWD/varlib/libppfit_xprof.so BENCH_ARGS="--fit align --nsub 1000 --nchan 256 --nbin 1024" \
  timeout -k 10 300 python tools/xprof.py > gpurun_out/xmprof_c4.txt 2>&1
rc=$?; tail -9 gpurun_out/xmprof_c4.txt; exit $rc

#!/bin/bash
# Section cycle profile of k_xspec_w2 (C2, 2500 sub-ints) from the
# PPF_XM_PROF build (tools/build_variant.sh x2prof -DPPF_XM_PROF=1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
PPFIT_LIB=$PWD/varlib/libppfit_x2prof.so XP_NAMES="convert+issue,fft1024,pairs,post-pass,tail,barrier1,writeout+barrier2,-" \
  timeout -k 10 300 python tools/xprof.py > gpurun_out/x2prof.txt 2>&1
rc=$?; tail -9 gpurun_out/x2prof.txt; exit $rc

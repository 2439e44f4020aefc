#!/bin/bash
# round 6: kernel statistics of the last build (C2, C4), kernel trace only
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/ks_final; mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/c2 -o ks --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > $out/c2.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/c4 -o ks --output-format csv -- python3 bench.py --fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 10 --warmup 2 --cpu-sample 0 > $out/c4.log 2>&1
rc=$?
find $out -name "*kernel_stats.csv" | head
exit $rc

#!/bin/bash
# Profiles: tools/prof.sh (kernel stats + FETCH/WRITE + SQ/f64 + TCC
# passes, each its own rocprofv3 run) for the named BASELINE configs.
# usage: tools/prof_round.sh TAG c2|c3|c5|c4|nb1000|nb1536|nb1023 ...
tag=${1:-a}; shift
for c in "$@"; do
  case $c in
    c2) a="";;
    c3) a="--fit full --nsub 10000";;
    c5) a="--fit scat --nchan 16384 --nbin 1024 --nsub 500";;
    c4) a="--fit align --nsub 1000 --nchan 256 --nbin 1024";;
    nb1000) a="--nbin 1000 --nsub 4000";;
    nb1536) a="--nbin 1536 --nsub 4000";;
    nb1023) a="--nbin 1023 --nsub 4000";;
  esac
  bash tools/prof.sh ${tag}_$c $a || exit 1
  echo "$c done" >> gpurun_out/prof_${tag}_status.txt
done
